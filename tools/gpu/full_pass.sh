# round-1 GPU pass b: parity tests, bench, kernel trace, PMC counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r1c}
mkdir -p $O
rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -rf --durations=15 > $O/gpu_tests.log 2>&1; echo "tests exit $?" >> $O/gpu_tests.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_trace.json 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_sq -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pmc_sq.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d $O/pmc_sq2 -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pmc_sq2.log 2>&1 || exit 1
echo ALLDONE
