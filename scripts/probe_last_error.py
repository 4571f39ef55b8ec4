"""Probe HIP's last-error semantics on this runtime (one GPU, seconds).

Does a failed call's error survive later successful calls and surface at the
next hipGetLastError()?  That is what makes an unchecked failure in a release
path (destructor, free) show up as a launch error in an unrelated object
later (hip_util.hpp: clear_release_error).  Also: does hipErrorNotReady from
hipEventQuery/hipStreamQuery count as a last error?
"""
import ctypes

hip = ctypes.CDLL("libamdhip64.so")
hip.hipGetErrorString.restype = ctypes.c_char_p


def name(e):
    return f"{e} ({hip.hipGetErrorString(e).decode()})"


def main():
    assert hip.hipSetDevice(0) == 0
    print("clean start:", name(hip.hipGetLastError()))
    bad = hip.hipSetDevice(9999)
    p = ctypes.c_void_p()
    ok = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20))
    ok2 = hip.hipMemset(p, 0, ctypes.c_size_t(1 << 20))
    print(f"failed call {name(bad)}, then hipMalloc {ok}, hipMemset {ok2}")
    print("last error after the successes:", name(hip.hipGetLastError()))
    print("and again:", name(hip.hipGetLastError()))
    hip.hipFree(p)
    # hipErrorNotReady: a stream kept busy by a long memset on a big buffer
    big = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(big), ctypes.c_size_t(1 << 31)) == 0
    s = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(s)) == 0
    for _ in range(8):
        hip.hipMemsetAsync(big, 1, ctypes.c_size_t(1 << 31), s)
    q = hip.hipStreamQuery(s)
    print("hipStreamQuery on a busy stream:", name(q))
    print("last error after it:", name(hip.hipGetLastError()))
    hip.hipStreamSynchronize(s)
    hip.hipStreamDestroy(s)
    hip.hipFree(big)
    hip.hipFree(ctypes.c_void_p(0x1234))  # an invalid free, as a release path might do
    print("after an invalid hipFree:", name(hip.hipGetLastError()))


if __name__ == "__main__":
    main()
