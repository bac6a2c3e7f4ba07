# Kernel traces + PMC passes (separate runs, no trace domains with --pmc) for the
# three renderers: bench.py (sphere cave), tools/bench_glsl.py, tools/bench_voxel.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-prof}
mkdir -p $O
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
run() {  # name, then the command after --
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${name}_trace -o run --output-format csv -- "$@" > $O/${name}_trace.log 2>&1 || return 1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/${name}_fetch -o run --output-format csv -- "$@" > $O/${name}_fetch.log 2>&1 || return 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/${name}_write -o run --output-format csv -- "$@" > $O/${name}_write.log 2>&1 || return 1
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/${name}_sq -o run --output-format csv -- "$@" > $O/${name}_sq.log 2>&1 || return 1
}
# ONLY=sphere|glsl|voxel limits the passes to one renderer
want() { [ -z "$ONLY" ] || [ "$ONLY" = "$1" ]; }
if want sphere; then run sphere python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline || exit 1; fi
if want glsl; then run glsl python3 tools/bench_glsl.py --no-cpu --steps 10 || exit 1; fi
if want voxel; then run voxel python3 tools/bench_voxel.py --no-cpu --steps 10 || exit 1; fi
echo ALLDONE
