"""Store-pattern microbenchmark driver (tools/store_bench.hip): TB/s per store shape on a 37759 x 768 fp32 matrix,
kernel time from HIP-graph replays.  usage: python tools/store_bench.py"""
import ctypes
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def timeit(fn, reps=20, per_graph=10):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per_graph):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / per_graph)
    return statistics.median(ts)


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "store_bench.so"))
    lib.store_bench.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    for M, N in [(37759, 768), (37759, 256), (37759, 1024)]:
        y = torch.zeros(M, N, device="cuda")
        out = []
        for pat in (0, 1, 2):
            t = timeit(lambda: lib.store_bench(pat, y.data_ptr(), M, N,
                                               ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
            out.append(f"pat{pat} {t:6.1f} us {M * N * 4 / t / 1e6:5.2f} TB/s")
        print(f"{M}x{N}: " + " | ".join(out), flush=True)
        ref = torch.empty_like(y)
        lib.store_bench(2, ref.data_ptr(), M, N, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        print("   pattern-2 coverage:", bool((ref.view(torch.int32)[:, 0] == torch.arange(M, device="cuda",
                                                                                       dtype=torch.int32)).all()))
    sys.stdout.flush()


if __name__ == "__main__":
    main()
