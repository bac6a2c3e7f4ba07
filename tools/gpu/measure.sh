# Measurement pass without the test suite: smoke(), the default bench line, the headline kernel
# trace + PMC passes (prof.sh), and the GLSL / voxel kernel traces + PMC passes.
#   /usr/local/graft/bin/gpurun --timeout 1500 -- "bash tools/gpu/measure.sh <tag>"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-measure}
O=gpurun_out/$T/pass
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
TAG=$T/prof bash tools/gpu/prof.sh || exit 1
TAG=$T/glsl bash tools/gpu/prof_glsl.sh || exit 1
TAG=$T/voxel bash tools/gpu/prof_voxel.sh || exit 1
echo measure done
