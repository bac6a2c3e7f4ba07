# SQ instruction counters of the 4K headline frame for each library in LIBS (A/B builds):
#   /usr/local/graft/bin/gpurun --timeout 600 -- "TAG=x LIBS=a.so,b.so bash tools/gpu/ab_pmc.sh"
# then: python tools/pmc_compare.py gpurun_out/x/pmc_*
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab_pmc}
mkdir -p $O
i=0
for L in ${LIBS//,/ }; do
  SFRT_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES \
    -d $O/pmc_$i -o run --output-format csv -- python tools/frame_loop.py 50 > $O/pmc_$i.log 2>&1 || exit 1
  echo "pmc_$i $L" >> $O/libs.txt
  i=$((i+1))
done
echo done
