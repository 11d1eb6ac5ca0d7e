"""Do two HIP streams of this process run kernels concurrently?  (C2 straggler analysis, r06: the
fleet's two class streams shared one hardware queue in the bench process -- profiles/r06/s3
kernel trace, Queue_Id.)  Launches one ~1 ms single-workgroup spin kernel (torch.cuda._sleep) on
each of two streams and times both: ~1 ms = concurrent, ~2 ms = serialized.  Cases: two torch
streams made first; two torch streams made after 6 others; two streams from
hipExtStreamCreateWithCUMask (all CUs: a stream with a CU mask gets a hardware queue of its own)."""
import ctypes
import time

import torch


def loaded_hip():
    """The HIP runtime this process already loaded (PyTorch's): never a second copy."""
    for line in open("/proc/self/maps"):
        if "libamdhip64.so" in line:
            return line.split()[-1]
    raise RuntimeError("libamdhip64 not loaded")


def cu_mask_stream(lib):
    s = ctypes.c_void_p()
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    words = (n_cu + 31) // 32
    mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
    rc = lib.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value)


def pair_ms(a, b, cycles):
    torch.cuda.synchronize()
    t = time.perf_counter()
    with torch.cuda.stream(a):
        torch.cuda._sleep(cycles)
    with torch.cuda.stream(b):
        torch.cuda._sleep(cycles)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3


def main():
    torch.cuda.init()
    cycles = 2_000_000
    s0 = torch.cuda.Stream()
    with torch.cuda.stream(s0):
        torch.cuda._sleep(cycles)  # warm-up
    torch.cuda.synchronize()
    t = time.perf_counter()
    with torch.cuda.stream(s0):
        torch.cuda._sleep(cycles)
    torch.cuda.synchronize()
    one = (time.perf_counter() - t) * 1e3
    print(f"one sleep: {one:.3f} ms")
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    print(f"two first torch streams: {pair_ms(a, b, cycles):.3f} ms")
    others = [torch.cuda.Stream() for _ in range(6)]
    for o in others:
        with torch.cuda.stream(o):
            torch.cuda._sleep(1000)
    c, d = torch.cuda.Stream(), torch.cuda.Stream()
    print(f"two torch streams after 6 others: {pair_ms(c, d, cycles):.3f} ms")
    lib = ctypes.CDLL(loaded_hip())
    e, f = cu_mask_stream(lib), cu_mask_stream(lib)
    print(f"two CU-mask streams: {pair_ms(e, f, cycles):.3f} ms")
    print(f"CU-mask stream + torch stream: {pair_ms(e, c, cycles):.3f} ms")


if __name__ == "__main__":
    main()
