# GLSL kernel: VALU/SALU counts and stall split (PMC passes), then per-wave work counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-glsl_sq}
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/sq -o run --output-format csv -- python3 tools/bench_glsl.py --no-cpu --steps 5 > $O/sq.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_SCA -d $O/sq2 -o run --output-format csv -- python3 tools/bench_glsl.py --no-cpu --steps 5 > $O/sq2.log 2>&1 || exit 1
python tools/instrument_glsl.py sfml-software-raytracer_amd/csrc/glsl_trace.hip && \
sed -i 's/-fvisibility=hidden //' sfml-software-raytracer_amd/Makefile && \
make -C sfml-software-raytracer_amd -j16 > $O/stats_build.log 2>&1 && \
timeout -k 10 300 python tools/glsl_work_counters.py > $O/stats.txt 2>&1
echo done
