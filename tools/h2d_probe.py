#!/usr/bin/env python3
"""Host-to-device DMA rate from pinned memory on the box, for the ingest line's ceiling: one stream
vs two, copy sizes of one C2 scan's compact record (1.42 MB) up to 64 MB."""
import time

import torch


def rate(size, total, streams):
    src = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    dst = torch.empty(total, dtype=torch.uint8, device="cuda")
    ss = [torch.cuda.Stream() for _ in range(streams)]
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k, o in enumerate(range(0, total, size)):
            with torch.cuda.stream(ss[k % streams]):
                dst[o:o + size].copy_(src[o:o + size], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    return total / dt / 1e9


def main():
    total = 1 << 31
    for size in (1_420_000, 4 << 20, 16 << 20, 64 << 20):
        for streams in (1, 2):
            print(f"copy {size / 1e6:7.2f} MB x {total // size:5d}, {streams} stream(s): {rate(size, total, streams):6.1f} GB/s",
                  flush=True)


if __name__ == "__main__":
    main()
