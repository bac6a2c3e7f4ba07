"""Which HIP allocation calls wait for work queued on an unrelated stream?  Each call runs with
~20 ms of work (torch.cuda._sleep) queued on another stream and reports its duration and whether
that work is still pending afterwards (profiles/r6u_hip_alloc_calls.txt: hipFree and hipHostFree
wait for the whole device; hipMalloc, hipHostMalloc, hipMallocAsync and hipFreeAsync do not --
the reason for sfrt_host.h RetiredHost and the stream-ordered growth paths).
    /usr/local/graft/bin/gpurun -- "python tools/gpu/probe_hostalloc.py"
"""
import ctypes, time
import torch
hip = ctypes.CDLL("libamdhip64.so")
b = torch.cuda.Stream()
torch.cuda.synchronize()
def busy_call(name, fn):
    with torch.cuda.stream(b):
        torch.cuda._sleep(40_000_000)
    t0 = time.perf_counter(); rc = fn(); t1 = time.perf_counter()
    print(f"{name}: rc={rc} {1e3 * (t1 - t0):.2f} ms, other stream still busy={not b.query()}", flush=True)
    torch.cuda.synchronize()
p = ctypes.c_void_p()
busy_call("hipHostMalloc 1 MB", lambda: hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20), 0))
busy_call("hipHostFree", lambda: hip.hipHostFree(p))
d = ctypes.c_void_p()
s = torch.cuda.Stream()
busy_call("hipMallocAsync 1 MB", lambda: hip.hipMallocAsync(ctypes.byref(d), ctypes.c_size_t(1 << 20), ctypes.c_void_p(s.cuda_stream)))
busy_call("hipFreeAsync", lambda: hip.hipFreeAsync(d, ctypes.c_void_p(s.cuda_stream)))
busy_call("hipMalloc 1 MB", lambda: hip.hipMalloc(ctypes.byref(d), ctypes.c_size_t(1 << 20)))
busy_call("hipFree", lambda: hip.hipFree(d))
busy_call("hipHostMalloc 1 MB again", lambda: hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20), 0))
busy_call("hipHostFree again", lambda: hip.hipHostFree(p))
