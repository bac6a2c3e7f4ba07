# One GPU pass for a tag: the -m gpu suite, smoke(), the default bench line, the kernel trace
# of the bench command and the PMC passes (tools/gpu/prof.sh), all under gpurun_out/<tag>/.
#   /usr/local/graft/bin/gpurun --timeout 1500 -- bash tools/gpu/round.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-round}
TAG=$T/pass bash tools/gpu/pass.sh || exit 1
TAG=$T/prof bash tools/gpu/prof.sh || exit 1
echo round done
