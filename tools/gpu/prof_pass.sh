# Round-1 measurement pass (TAG names it) measurement pass: default bench line, then kernel trace of the same
# command and separate PMC passes (short runs) for the three renderers.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r1j}
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/sphere_trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/sphere_trace.log 2>&1 || exit 1
pmc() {  # name, counters..., then -- command
  local name=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done; shift
  timeout -s KILL 120 rocprofv3 --pmc "${ctr[@]}" -d $O/$name -o run --output-format csv -- "$@" > $O/$name.log 2>&1
}
SPH="python3 bench.py --no-cpu-baseline --settle 0 --steps 5 --warmup 1 --no-extra"
pmc sphere_fetch FETCH_SIZE -- $SPH || exit 1
pmc sphere_write WRITE_SIZE -- $SPH || exit 1
pmc sphere_sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- $SPH || exit 1
pmc sphere_sq2 SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -- $SPH || exit 1
VOX="python3 tools/bench_voxel.py --no-cpu --steps 10"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/voxel_trace -o run --output-format csv -- $VOX > $O/voxel_trace.log 2>&1 || exit 1
pmc voxel_fetch FETCH_SIZE -- $VOX || exit 1
pmc voxel_write WRITE_SIZE -- $VOX || exit 1
pmc voxel_sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- $VOX || exit 1
echo ALLDONE
