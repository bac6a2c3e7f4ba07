set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_r1a.json 2> gpurun_out/bench_r1a.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1a -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_r1a_prof.json 2> gpurun_out/bench_r1a_prof.err
echo EXIT $?
