# Does RCCL take two ranks on ONE device here?  (the one-GPU box's tests use peer
# copies for devices [0] * n and one-rank RCCL; this is the evidence for that choice.)
#  (1) torch.distributed "nccl" with two processes on cuda:0 (tools/gpu/nccl_same_device.py);
#  (2) ncclCommInitAll over devices [0, 0] (what sfrt_multi's RCCL transport would call).
# Each under its own time limit; NCCL_DEBUG=WARN keeps RCCL's own reason in the log.
#   /usr/local/graft/bin/gpurun --timeout 600 -- "TAG=r6d bash tools/gpu/rccl_same_device.sh"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-rccl_same}
mkdir -p $O
NCCL_DEBUG=WARN timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr 127.0.0.1 --master-port 29531 tools/gpu/nccl_same_device.py > $O/torch_two_ranks.log 2>&1
rc=$?
echo "exit $rc" >> $O/torch_two_ranks.log
[ $rc -ge 124 ] && exit 1  # a time limit or a signal: nothing more on the GPU in this call
NCCL_DEBUG=WARN timeout -k 10 120 python -c "
import ctypes
lib = ctypes.CDLL('librccl.so.1')
lib.ncclGetErrorString.restype = ctypes.c_char_p
comms = (ctypes.c_void_p * 2)()
devs = (ctypes.c_int * 2)(0, 0)
rc = lib.ncclCommInitAll(comms, 2, devs)
print('ncclCommInitAll(2, [0, 0]) ->', rc, lib.ncclGetErrorString(rc).decode())
if rc == 0:
    for c in comms:
        lib.ncclCommDestroy(ctypes.c_void_p(c))
" > $O/comm_init_all_0_0.log 2>&1
rc=$?
echo "exit $rc" >> $O/comm_init_all_0_0.log
[ $rc -ge 124 ] && exit 1
echo done
