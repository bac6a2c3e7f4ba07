# Instruction-cache PMC passes of the three kernels (SQC_ICACHE_*, SQ_IFETCH):
#   /usr/local/graft/bin/gpurun --timeout 600 -- "TAG=r6ic bash tools/gpu/prof_icache.sh"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-icache}
mkdir -p $O
timeout -s KILL 60 rocprofv3 --list-avail > $O/list_avail.txt 2>&1 || exit 1
grep -i "icache\|ifetch" $O/list_avail.txt > $O/icache_counters.txt || true
C=${COUNTERS:-"SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH"}
timeout -s KILL 90 rocprofv3 --pmc $C -d $O/sphere -o run --output-format csv -- python tools/frame_loop.py 50 > $O/sphere.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $C -d $O/glsl -o run --output-format csv -- python tools/bench_glsl.py --no-cpu --steps 20 --set bench > $O/glsl.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $C -d $O/voxel -o run --output-format csv -- python tools/bench_voxel.py --no-cpu --steps 20 --set bench > $O/voxel.log 2>&1 || exit 1
echo done
