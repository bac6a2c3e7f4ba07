# Full round pass on the current tree: the -m gpu suite, smoke(), the default bench line, the
# headline kernel trace (tools/gpu/pass.sh) and the kernel traces + PMC passes of all three
# kernels (tools/gpu/prof_all.sh), under gpurun_out/$TAG/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:?}
TAG=$T/pass bash tools/gpu/pass.sh || exit 1
TAG=$T/prof bash tools/gpu/prof_all.sh || exit 1
echo all done
