set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5o
mkdir -p $O
for i in 1 2; do
  for v in 0 1; do
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python bench.py --headline-only --no-cpu-baseline --steps 400 --warmup 50 > $O/kernarg_${v}_$i.json 2> $O/kernarg_${v}_$i.err || exit 1
  done
done
echo done
