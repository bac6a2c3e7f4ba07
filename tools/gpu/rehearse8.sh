# bench.py --gpus 8 rehearsed on one GPU (every rank on cuda:0 over gloo; test only): the N = 8
# body, including the 16384^2 line and the c_abi_multi child over [0]*8, which only N = 8 runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-rehearse8}
mkdir -p $O
timeout -k 10 ${TMO:-900} python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --rehearse --bands ${BANDS:-equal} \
  --steps 6 --warmup 2 --settle 0 --also-steps 20 --also-warmup 5 --also-settle 0 \
  --no-cpu-baseline > $O/bench8.json 2> $O/bench8.err
rc=$?
echo "exit $rc" >> $O/bench8.err
exit $rc
