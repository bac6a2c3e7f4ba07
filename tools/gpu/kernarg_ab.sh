# Headline with the kernel arguments in host memory (0), device memory (1) and the runtime's default (unset),
# alternating (profiles/ab/r5_ab9):  /usr/local/graft/bin/gpurun -- "bash tools/gpu/kernarg_ab.sh"
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-kernarg}
mkdir -p $O
for i in 1 2; do
  for v in unset 1 0; do
    if [ $v = unset ]; then
      timeout -k 10 200 python bench.py --headline-only --no-cpu-baseline --steps 400 --warmup 50 > $O/kernarg_${v}_$i.json 2> $O/kernarg_${v}_$i.err || exit 1
    else
      HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python bench.py --headline-only --no-cpu-baseline --steps 400 --warmup 50 > $O/kernarg_${v}_$i.json 2> $O/kernarg_${v}_$i.err || exit 1
    fi
  done
done
echo done
