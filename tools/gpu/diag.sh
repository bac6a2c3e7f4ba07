# Diagnostic builds on the GPU: per-tile timeline (-DSFRT_EXP=16) and visit counters (-DSFRT_EXP=32)
#   /usr/local/graft/bin/gpurun --timeout 600 -- "TAG=r3d bash tools/gpu/diag.sh"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-diag}
mkdir -p $O
P=sfml-software-raytracer_amd
SFRT_LIB=$P/build_x16/libsfrt.so timeout -k 10 200 python -u tools/tile_timeline.py > $O/tile_timeline_4k.txt 2>&1 || exit 1
SFRT_LIB=$P/build_x16/libsfrt.so timeout -k 10 200 python -u tools/tile_timeline.py --1080 > $O/tile_timeline_1080p.txt 2>&1 || exit 1
SFRT_LIB=$P/build_x32/libsfrt.so timeout -k 10 200 python -u tools/visit_counts.py > $O/visit_counts.txt 2>&1 || exit 1
echo done
