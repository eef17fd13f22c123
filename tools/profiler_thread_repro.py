"""Isolation check for the rocprofv3 crash seen with the many-windows BA leg (development tool).

Under `rocprofv3 --kernel-trace`, 16 host threads that each launch short kernels on their own
stream — here plain PyTorch kernels, none of libmage_hot.so — exercise the same launch pattern
as bench.py's many-windows leg (16 BundlerLib instances, one HIP stream + host thread each).
If this segfaults under the profiler and runs clean without it, the fault is the profiler's.

  rocprofv3 --kernel-trace --stats -d <dir> -o run -- python3 tools/profiler_thread_repro.py
"""
import concurrent.futures as cf
import sys
import time

import torch


def work(i, seconds):
    s = torch.cuda.Stream()
    x = torch.randn(256, 256, device="cuda")
    n, t0 = 0, time.perf_counter()
    with torch.cuda.stream(s):
        while time.perf_counter() - t0 < seconds:
            for _ in range(12):  # ~12 short launches per readback, like one BA trial
                x = torch.tanh(x * 0.5 + 0.1)
            _ = float(x[0, 0].item())
            n += 1
    return n


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    seconds = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
    torch.cuda.init()
    with cf.ThreadPoolExecutor(threads) as ex:
        counts = list(ex.map(lambda i: work(i, seconds), range(threads)))
    print({"threads": threads, "readbacks": sum(counts)}, flush=True)


if __name__ == "__main__":
    main()
