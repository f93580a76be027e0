"""Command line for the homework suite -- the reference's per-homework drivers as subcommands.

  python -m cme213_sp18_amd.suite sum      [--n 30000000]                 (hw1 main_q1)
  python -m cme213_sp18_amd.suite radix    [--n 50000000] [--bits 8] [--blocks 8] [--sweep]   (hw1 main_q2)
  python -m cme213_sp18_amd.suite shift    [--text FILE] [--doublings 8]   (hw2 main_q1)
  python -m cme213_sp18_amd.suite pagerank [--quick]                       (hw2 main_q2)
  python -m cme213_sp18_amd.suite stencil  [-g] [-b] [-s] [--params params.in]   (hw3 main)
  python -m cme213_sp18_amd.suite create_cipher TEXT PERIOD                (hw4 create_cipher)
  python -m cme213_sp18_amd.suite solve_cipher CIPHER                      (hw4 solve_cipher)

Every GPU result is checked against the CPU oracle, as the reference drivers do.
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import numpy as np


def _cuda():
    import torch

    if not torch.cuda.is_available():
        sys.exit("this subcommand needs a GPU")
    return torch


def cmd_sum(a):
    from . import hw1

    v = hw1.init_sum_input(a.n)
    hw1.sum_even_odd_serial(v[:1000])
    hw1.sum_even_odd_parallel(v)  # OpenMP thread-pool start-up outside the timing
    t0 = time.perf_counter()
    s = hw1.sum_even_odd_serial(v)
    t1 = time.perf_counter()
    p = hw1.sum_even_odd_parallel(v)
    t2 = time.perf_counter()
    res = {"n": a.n, "serial_ms": (t1 - t0) * 1e3, "openmp_ms": (t2 - t1) * 1e3, "sums": s, "match": s == p}
    try:
        torch = _cuda()
        d = torch.from_numpy(v.view(np.int32)).cuda()
        out = torch.empty(2, dtype=torch.int64, device=d.device)  # allocated once, outside the timing
        hw1.sum_even_odd_gpu(d, out)
        from ._dev import EventTimer

        reps = 20  # device time per call, averaged over back-to-back launches (host overhead overlapped)
        with EventTimer() as t:
            for _ in range(reps):
                g = hw1.sum_even_odd_gpu(d, out)
        ms = t.ms / reps
        res.update(gpu_ms=ms, gpu_match=tuple(g.cpu().tolist()) == s, gpu_gbps=4 * a.n / (ms * 1e-3) / 1e9)
        if a.hbm:  # the same kernel on an input 8x the 256 MB MALL: an HBM-bound number
            big = torch.randint(0, 2**31 - 1, (a.hbm,), dtype=torch.int32, device=d.device)
            hw1.sum_even_odd_gpu(big, out)
            with EventTimer() as t:
                for _ in range(5):
                    gb = hw1.sum_even_odd_gpu(big, out)
            ms_b = t.ms / 5
            bb = big.to(torch.int64)
            ok_b = gb.tolist() == [int(bb[bb % 2 == 0].sum()), int(bb[bb % 2 == 1].sum())]
            res.update(hbm_n=a.hbm, hbm_ms=ms_b, hbm_gbps=4 * a.hbm / (ms_b * 1e-3) / 1e9, hbm_match=ok_b)
    except SystemExit:
        pass
    print(json.dumps(res))
    return 0 if res["match"] and res.get("gpu_match", True) and res.get("hbm_match", True) else 1


def cmd_radix(a):
    from . import hw1

    keys = np.random.default_rng(0).integers(0, 2**32, a.n, dtype=np.uint64).astype(np.uint32)
    # the reference's baseline is C++ std::sort (hw1code/main_q2.cpp:249-256); numpy's SIMD sort is listed too
    t0 = time.perf_counter()
    ref = hw1.std_sort(keys)
    std_ms = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    np_ref = np.sort(keys)
    np_ms = (time.perf_counter() - t0) * 1e3
    assert np.array_equal(ref, np_ref)
    hw1.radix_sort_parallel(keys, a.bits, a.blocks)  # warm the pool and the pages
    rows = []
    if a.sweep:  # main_q2.cpp:282-309 (-DQUESTION6): threads x blocks
        import os

        for blocks in (1, 2, 4, 8, 16, 32, 64):
            t0 = time.perf_counter()
            out = hw1.radix_sort_parallel(keys, a.bits, blocks)
            rows.append({"threads": os.environ.get("OMP_NUM_THREADS", "default"), "blocks": blocks,
                         "ms": (time.perf_counter() - t0) * 1e3, "ok": bool(np.array_equal(out, ref))})
    t0 = time.perf_counter()
    ser = hw1.radix_sort_serial(keys)
    t1 = time.perf_counter()
    par = hw1.radix_sort_parallel(keys, a.bits, a.blocks)
    t2 = time.perf_counter()
    lsd = hw1.radix_sort_lsd(keys)
    t3 = time.perf_counter()
    res = {"n": a.n, "std_sort_ms": std_ms, "np_sort_ms": np_ms, "serial_ms": (t1 - t0) * 1e3,
           "openmp_ms": (t2 - t1) * 1e3, "openmp_lsd_ms": (t3 - t2) * 1e3,
           "serial_ok": bool(np.array_equal(ser, ref)), "openmp_ok": bool(np.array_equal(par, ref)),
           "openmp_lsd_ok": bool(np.array_equal(lsd, ref)), "sweep": rows}
    try:
        torch = _cuda()
        from ._dev import EventTimer

        d = torch.from_numpy(keys.view(np.int32)).cuda()
        srt = hw1.GpuRadixSorter(a.n)
        w = d.clone()
        srt.sort_(w)
        reps = 10  # device time per sort, averaged (each rep re-sorts a fresh copy; the copies are timed apart)
        ms = 0.0
        for _ in range(reps):
            w.copy_(d)
            with EventTimer() as t:
                srt.sort_(w)
            ms += t.ms / reps
        res.update(gpu_ms=ms, gpu_ok=bool(np.array_equal(w.cpu().numpy().view(np.uint32), ref)),
                   gpu_mkeys_per_s=a.n / (ms * 1e-3) / 1e6)
    except SystemExit:
        pass
    print(json.dumps(res))
    return 0 if res["serial_ok"] and res["openmp_ok"] and res.get("gpu_ok", True) else 1


def cmd_shift(a):
    from . import hw2, hw4

    _cuda()
    text = hw4.read_text(a.text)  # default: the reference's Moby Dick (tests/fixtures)
    print(f"{'bytes':>12} " + " ".join(f"{'w=' + str(w) + ' GB/s':>12}" for w in hw2.SHIFT_WIDTHS))
    rows = []
    for d in range(a.doublings + 1):
        r = hw2.benchmark_shift(hw2.doubled_text(text, d), shift=a.shift, reps=a.reps)
        rows.append(r)
        print(f"{r['bytes']:>12} " + " ".join(f"{r['gbps'][w]:>12.1f}" for w in hw2.SHIFT_WIDTHS), flush=True)
    if a.json:
        print(json.dumps(rows))
    return 0


def cmd_pagerank(a):
    from . import hw2

    _cuda()
    nodes = [1 << 15, 1 << 17] if a.quick else [1 << k for k in range(15, 21)]
    edges = [2, 10, 19] if a.quick else list(range(2, 20))
    rows = hw2.benchmark_pagerank(nodes, edges, variant=a.variant)
    hdr = "edges \\ nodes"
    print(f"{'GB/s':>60}\n{hdr:>15}" + "".join(f"{n:>15}" for n in nodes))
    for e in edges:
        print(f"{e:>15}" + "".join(f"{r['gbps']:>15.2f}" for r in rows if r["avg_edges"] == e), flush=True)
    bad = sum(r["mismatches"] for r in rows)
    if a.json:
        print(json.dumps(rows))
    return 1 if bad else 0


def cmd_stencil(a):
    from . import hw3

    _cuda()
    p = hw3.SimParams.from_file(a.params) if a.params else hw3.SimParams(a.nx, a.ny, 1.0, 1.0, a.iters, a.order)
    chosen = ([v for v, f in (("global", a.g), ("block", a.b), ("shared", a.s), ("vec", a.v), ("shared2", a.t)) if f]
              or ["global", "block", "shared", "vec", "shared2"])
    g0 = hw3.init_grid(p)
    t0 = time.perf_counter()
    ref = hw3.cpu_computation(g0, p)
    cpu_ms = (time.perf_counter() - t0) * 1e3
    print(f"order={p.order} grid={p.nx}x{p.ny} iters={p.iters}  CPU {cpu_ms:.1f} ms")
    rc = 0
    res = {"cpu_ms": cpu_ms}
    for v in chosen:
        hw3.gpu_computation(g0, hw3.SimParams(p.nx, p.ny, p.lx, p.ly, min(p.iters, 2), p.order), v)  # warm
        out, ms = hw3.gpu_computation(g0, p, v)
        err = hw3.check_errors(ref, out)
        gbps = p.calc_bytes() / (ms * 1e-3) / 1e9          # the reference's model (every tap a read)
        gbps_act = p.compulsory_bytes() / (ms * 1e-3) / 1e9  # bytes an ideal kernel moves: read grid, write grid
        print(f"{v:>8}: {ms:10.3f} ms  model {gbps:8.1f} GB/s  actual {gbps_act:8.1f} GB/s  "
              f"mismatches={err['mismatches']} L2Ref={err['l2ref']:.6g} LInf={err['linf']:.3g} "
              f"L2Err={err['l2err']:.3g}", flush=True)
        res[v] = {"ms": ms, "gbps": gbps, "gbps_actual": gbps_act, **err}
        rc |= err["mismatches"] != 0
    if a.json:
        print(json.dumps(res))
    return int(rc)


def cmd_create_cipher(a):
    from . import hw4

    _cuda()
    text = hw4.read_text(None if a.text == "-" else a.text)
    clean = hw4.sanitize(text)
    print("\nBefore ciphering!\n")
    g = hw4.letter_frequency_gpu(clean)
    c = hw4.letter_frequency_cpu(text)
    ok = len(g) == len(c) and all(abs(x - y) < 1e-14 for x, y in zip(g, c))
    for i, f in enumerate(g):
        print(f"{i} {f:f}")
    print("TEST PASSED" if ok else "TEST FAILED")
    shifts = hw4.make_shifts(a.period, a.seed)
    print(f"\nEncryption key: {hw4.key_string(shifts)}")
    cipher = hw4.apply_shift(clean, shifts, 1, not a.no_wrap)
    print("After ciphering!\n")
    for i, f in enumerate(hw4.letter_frequency_gpu(cipher) if not a.no_wrap else []):
        print(f"{i} {f:f}")
    open(a.out, "wb").write(cipher.cpu().numpy().tobytes())
    return 0 if ok else 1


def cmd_solve_cipher(a):
    from . import hw4

    _cuda()
    plain, shifts, k = hw4.solve_cipher(open(a.cipher, "rb").read(), a.max_period, not a.no_wrap)
    print(f"keyLength: {k}\n\nEncryption key: {hw4.key_string(shifts)}")
    open(a.out, "wb").write(plain.cpu().numpy().tobytes())
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m cme213_sp18_amd.suite")
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("sum")
    s.add_argument("--n", type=int, default=30_000_000)
    s.add_argument("--hbm", type=int, default=0,
                   help="also time the GPU kernel on this many random int32 (e.g. 536870912 = 2 GB > the 256 MB MALL)")
    s = sub.add_parser("radix")
    s.add_argument("--n", type=int, default=4_000_000)  # main_q2.cpp:14
    s.add_argument("--bits", type=int, default=8)
    s.add_argument("--blocks", type=int, default=8)
    s.add_argument("--sweep", action="store_true")
    s = sub.add_parser("shift")
    s.add_argument("--text")
    s.add_argument("--doublings", type=int, default=8)
    s.add_argument("--shift", type=int, default=3)
    s.add_argument("--reps", type=int, default=20)
    s.add_argument("--json", action="store_true")
    s = sub.add_parser("pagerank")
    s.add_argument("--quick", action="store_true")
    s.add_argument("--variant", type=int, default=3,
                   help="3: pre-multiplied gather (default); 0: thread per node; 1: 8 lanes per node; 2: auto (0)")
    s.add_argument("--json", action="store_true")
    s = sub.add_parser("stencil")
    s.add_argument("-g", action="store_true", help="global-memory kernel")
    s.add_argument("-b", action="store_true", help="register-blocked (loop) kernel")
    s.add_argument("-s", action="store_true", help="LDS-tiled kernel")
    s.add_argument("-v", action="store_true", help="16-byte-vector register-window kernel")
    s.add_argument("-t", action="store_true",
                   help="LDS-tiled kernel with temporal blocking: two time steps per sweep of the grid (order 8)")
    s.add_argument("--params")
    s.add_argument("--nx", type=int, default=4096)
    s.add_argument("--ny", type=int, default=4096)
    s.add_argument("--iters", type=int, default=400)
    s.add_argument("--order", type=int, default=8)
    s.add_argument("--json", action="store_true")
    s = sub.add_parser("create_cipher")
    s.add_argument("text", help="plaintext file (.gz ok); '-' = the shipped Moby Dick")
    s.add_argument("period", type=int)
    s.add_argument("--seed", type=int, default=123)
    s.add_argument("--no-wrap", action="store_true", help="reference byte-add semantics")
    s.add_argument("--out", default="cipher_text.txt")
    s = sub.add_parser("solve_cipher")
    s.add_argument("cipher")
    s.add_argument("--max-period", type=int, default=256)
    s.add_argument("--no-wrap", action="store_true")
    s.add_argument("--out", default="plain_text.txt")
    a = ap.parse_args(argv)
    return globals()[f"cmd_{a.cmd}"](a)


if __name__ == "__main__":
    sys.exit(main())
