"""What do HIP calls return for the handle of a stream the caller already destroyed?  The renderers
remember the stream of a chain's last launch (sfrt_sched.h TileSched::last_stream) and later
synchronise with it or free on it; a caller may have destroyed that stream in between.
    /usr/local/graft/bin/gpurun -- "python tools/gpu/probe_dead_stream.py"
"""
import ctypes

hip = ctypes.CDLL("libamdhip64.so")
vp = ctypes.c_void_p


def name(e):
    hip.hipGetErrorName.restype = ctypes.c_char_p
    return f"{e} ({hip.hipGetErrorName(e).decode()})"


def main():
    s = vp()
    assert hip.hipStreamCreate(ctypes.byref(s)) == 0
    p = vp()
    assert hip.hipMallocAsync(ctypes.byref(p), ctypes.c_size_t(1 << 20), s) == 0
    assert hip.hipStreamSynchronize(s) == 0
    print("live stream: query", name(hip.hipStreamQuery(s)), flush=True)
    assert hip.hipStreamDestroy(s) == 0
    print("destroyed stream: query", name(hip.hipStreamQuery(s)), flush=True)
    print("destroyed stream: synchronize", name(hip.hipStreamSynchronize(s)), flush=True)
    print("destroyed stream: free_async", name(hip.hipFreeAsync(p, s)), flush=True)
    q = vp()
    assert hip.hipStreamCreate(ctypes.byref(q)) == 0
    print("a new stream reuses the handle:", q.value == s.value, flush=True)
    print("device synchronize", name(hip.hipDeviceSynchronize()), flush=True)


if __name__ == "__main__":
    main()
