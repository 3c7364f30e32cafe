#!/usr/bin/env python3
"""Pinned host-to-device copy rate by chunk size and number of concurrent copy streams (tools only):
is one stream's upload (the pipelined schedule's shape) below what the link takes with two?
Prints one JSON line."""
import json
import time

import torch


def main():
    n = 1 << 30
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h.fill_(1)
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(4)]
    res = {}
    for chunk_mb in (8, 25, 64):
        c = chunk_mb << 20
        k = n // c
        for ns in (1, 2, 3):
            best = 1e9
            for _ in range(4):
                torch.cuda.synchronize()
                t = time.perf_counter()
                for i in range(k):
                    if ns == 1:
                        with torch.cuda.stream(streams[0]):
                            d[i * c:(i + 1) * c].copy_(h[i * c:(i + 1) * c], non_blocking=True)
                    else:  # each chunk split across ns streams
                        p = c // ns
                        for j in range(ns):
                            a = i * c + j * p
                            b = (i + 1) * c if j == ns - 1 else a + p
                            with torch.cuda.stream(streams[j]):
                                d[a:b].copy_(h[a:b], non_blocking=True)
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t)
            res[f"{chunk_mb}MiB_x{ns}"] = round(k * c / best / 1e9, 2)
    # the pipeline's surroundings: downloads beside the uploads, and 16 host threads hashing other
    # pinned buffers (the MD5 pool's memory traffic) beside them
    import hashlib
    import threading

    c = 25 << 20
    k = n // c
    dn = torch.empty(n // 2, dtype=torch.uint8, pin_memory=True)
    dsrc = torch.ones(n // 2, dtype=torch.uint8, device="cuda")
    bufs = [torch.empty(256 << 20, dtype=torch.uint8, pin_memory=True).numpy() for _ in range(16)]
    stop = [False]

    def hasher(b):
        while not stop[0]:
            hashlib.md5(b).digest()

    def run(d2h):
        best = 1e9
        for _ in range(4):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for i in range(k):
                with torch.cuda.stream(streams[0]):
                    d[i * c:(i + 1) * c].copy_(h[i * c:(i + 1) * c], non_blocking=True)
                if d2h and i % 2 == 0:
                    j = (i // 2) % (n // 2 // c)
                    with torch.cuda.stream(streams[1]):
                        dn[j * c:(j + 1) * c].copy_(dsrc[j * c:(j + 1) * c], non_blocking=True)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t)
        return round(k * c / best / 1e9, 2)

    res["25MiB_x1_with_d2h"] = run(True)
    th = [threading.Thread(target=hasher, args=(b,)) for b in bufs]
    for x in th:
        x.start()
    time.sleep(0.2)
    res["25MiB_x1_with_16_md5_threads"] = run(False)
    res["25MiB_x1_with_d2h_and_16_md5_threads"] = run(True)
    stop[0] = True
    for x in th:
        x.join()
    del bufs
    # the e2e batch's sources: 64 separate pinned file buffers of 106 MB (10 min of 16-bit stereo),
    # uploaded in 32-MiB chunks one after another; then the same beside a compute-bound kernel
    files = [torch.empty(106 << 20, dtype=torch.uint8, pin_memory=True) for _ in range(24)]
    for f in files:
        f.fill_(2)
    c = 32 << 20

    def files_up():
        torch.cuda.synchronize()
        t = time.perf_counter()
        tot = 0
        with torch.cuda.stream(streams[0]):
            for f in files:
                for o in range(0, f.numel(), c):
                    m = min(c, f.numel() - o)
                    d[:m].copy_(f[o:o + m], non_blocking=True)
                    tot += m
        streams[0].synchronize()
        return tot / (time.perf_counter() - t) / 1e9

    res["files_32MiB_x1"] = round(max(files_up() for _ in range(3)), 2)
    a = torch.randn(8192, 8192, device="cuda")
    busy = [True]

    def compute():
        with torch.cuda.stream(streams[2]):
            while busy[0]:
                for _ in range(8):
                    torch.mm(a, a)
                streams[2].synchronize()

    tc = threading.Thread(target=compute)
    tc.start()
    time.sleep(0.3)
    res["files_32MiB_x1_beside_gemm"] = round(max(files_up() for _ in range(3)), 2)
    busy[0] = False
    tc.join()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
