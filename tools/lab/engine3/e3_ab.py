"""Lab A/B: one decode layer as the engine-v3 persistent launch (tools/lab/engine3/engine3.hip) against the product's
five per-op launches, at a rank geometry, in ONE process on one GPU (VERDICT r5 "Next round" item 1, stop rule
<= 0.9x the per-op graph at 7B TP = 1 and at the 7B TP = 8 rank).

usage: python tools/lab/engine3/e3_ab.py [--geom 7b1|7b8] [--layers 32] [--pos 2200] [--check] [--floor]

Both sides get `layers` distinct weight / KV copies (int4-g128 by the product quantizer; the group the product fits to
a shard's K), HIP-graph replays of all layers back to back, best of 3 x 10 replays; printed as us per layer. --check
compares every engine op output of layer 0 with torch / product references of the same math (the engine skips RoPE
and does not reproduce the product's summation order: tolerances, not bit equality). --floor adds the engine with its
consumers computing nothing (transport + hand-off floor).
"""

import argparse
import os
import ctypes
import math
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[3]
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO)]

from lit_gpt import ops  # noqa: E402

GEOMS = {"7b1": (4096, 32, 32, 11008, 1), "7b8": (4096, 32, 32, 11008, 8)}
SLOT = 17408


def q4(N, K, dev):
    from lit_gpt.quantize import _fit_group

    g = _fit_group(K, 128)
    qw, sc = ops.quantize(torch.randn(N, K, device=dev) * 0.02, ops.FMT_Q4G, g)
    return qw, sc, g


def rows_per_unit(K, G, dual):
    rb = K // 2 + (K // G) * 2
    r = SLOT // (2 * rb if dual else rb)
    r = min(r, 8 if dual else 16)
    if ((K // G) * 2) % 4:
        r -= r % 2  # dword DMA of the scales needs 4-byte aligned unit starts
    return r


def time_graph(fn, layers, reps=10):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            g.replay()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / (reps * layers))
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--geom", default="7b1")
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--pos", type=int, default=2200)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--floor", action="store_true")
    ap.add_argument("--trace", action="store_true", help="per-op event times of one launch (static ranges)")
    ap.add_argument("--lib", default="liblga_engine3.so", help="engine build under tools/_ab (slot / consumer count)")
    ap.add_argument("--esplits", type=int, default=1, help="the engine's attention splits = this x the product's")
    args = ap.parse_args()
    dev = torch.device("cuda")
    C, H, G, I, tp = GEOMS[args.geom]
    hs, L, pos = 128, args.layers, args.pos
    Hr, Gr, Ir = H // tp, max(1, G // tp), I // tp
    Kp = Hr * hs
    S = pos + 64
    Nq = (Hr + 2 * Gr) * hs
    W = [dict(qkv=q4(Nq, C, dev), proj=q4(C, Kp, dev), fc1=q4(Ir, C, dev), fc2=q4(Ir, C, dev), down=q4(C, Ir, dev),
              kc=torch.randn(Gr, S, hs, device=dev).bfloat16(), vc=torch.randn(Gr, S, hs, device=dev).bfloat16(),
              n1=(1.0 + 0.1 * torch.randn(C, device=dev)).bfloat16(),
              n2=(1.0 + 0.1 * torch.randn(C, device=dev)).bfloat16()) for _ in range(L)]
    x0 = torch.randn(C, device=dev).bfloat16()
    p = torch.tensor([pos], device=dev)
    splits = ops.decode_splits(Gr, Hr // Gr, hs, S)
    scale = 1.0 / math.sqrt(hs)

    # ---- the product: five launches per layer ----
    x = x0.clone()
    qkv = torch.empty(Nq, device=dev, dtype=torch.bfloat16)
    y = torch.empty(Kp, device=dev, dtype=torch.bfloat16)
    o = torch.empty(C, device=dev, dtype=torch.bfloat16)
    g = torch.empty(Ir, device=dev, dtype=torch.bfloat16)
    cos, sin = torch.ones(S, hs, device=dev), torch.zeros(S, hs, device=dev)
    ws = ops.AttentionWorkspace(1, Hr, Gr, hs, splits, dev)

    def f_layer():
        for w in W:
            ops.q4_gemv(x, *w["qkv"][:2], Nq, C, w["qkv"][2], 0, norm_weight=w["n1"], out=qkv)
            ops.attention_decode_fused(qkv.view(1, -1), w["kc"], w["vc"], p, p, cos, sin, Hr, Gr, hs, hs, scale,
                                       splits, workspace=ws, out=y.view(1, -1))
            ops.q4_gemv(y, *w["proj"][:2], C, Kp, w["proj"][2], 0, residual=x, out=o)
            ops.q4_gemv_swiglu(o, *w["fc1"][:2], *w["fc2"][:2], Ir, C, w["fc1"][2], 0, norm_weight=w["n2"], out=g)
            ops.q4_gemv(g, *w["down"][:2], C, Ir, w["down"][2], 0, residual=o, out=x)

    # ---- the engine ----
    lib = ctypes.CDLL(str(REPO / "tools" / "_ab" / args.lib))
    global SLOT
    SLOT = lib.lga_e3_slot_bytes()
    ncons = lib.lga_e3_consumers()
    esplits = splits * args.esplits
    lib.lga_e3_launch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    assert lib.lga_e3_layer_bytes() == 14 * 8
    ptrs = []
    for w in W:
        ptrs += [w["qkv"][0].data_ptr(), w["qkv"][1].data_ptr(), w["proj"][0].data_ptr(), w["proj"][1].data_ptr(),
                 w["fc1"][0].data_ptr(), w["fc1"][1].data_ptr(), w["fc2"][0].data_ptr(), w["fc2"][1].data_ptr(),
                 w["down"][0].data_ptr(), w["down"][1].data_ptr(), w["kc"].data_ptr(), w["vc"].data_ptr(),
                 w["n1"].data_ptr(), w["n2"].data_ptr()]
    layers_dev = torch.tensor(ptrs, dtype=torch.int64, device=dev)
    gq, gp, gi = W[0]["qkv"][2], W[0]["proj"][2], W[0]["down"][2]
    ru = [rows_per_unit(C, gq, False), 0, rows_per_unit(Kp, gp, False), rows_per_unit(C, gq, True),
          rows_per_unit(Ir, gi, False)]
    units = [-(-Nq // ru[0]), Gr * esplits, -(-C // ru[2]), -(-Ir // ru[3]), -(-C // ru[4])]
    offs = [0]
    for n in (Nq, Kp, C, Ir):
        offs.append(offs[-1] + ((n + 63) // 64) * 64)
    stride = offs[-1] + ((C + 63) // 64) * 64
    act = torch.zeros(L * stride, device=dev, dtype=torch.bfloat16)
    ews = torch.zeros(L * Hr * esplits * (hs + 4), device=dev, dtype=torch.float32)
    ctr = torch.zeros(lib.lga_e3_counter_words(L, Gr), device=dev, dtype=torch.int32)
    err = torch.zeros(64 + 256 * 8 * 128, device=dev, dtype=torch.int32)  # word 0: error bits; then per-wave records
    n_cu = ops.num_cus()
    assert Hr == Gr, "the lab engine covers one query head per group"
    print(f"{args.geom}: rank H={Hr} G={Gr} I={Ir} Kp={Kp} splits={splits} rows/unit {ru} units {units} "
          f"LDS {lib.lga_e3_lds_bytes()} B, {n_cu} CUs; engine: {args.lib} slot {SLOT} B, {ncons} consumers, "
          f"{esplits} splits", flush=True)

    trace = torch.zeros(256 + 5 * L * n_cu * 32, device=dev, dtype=torch.int64)

    def make_args(compute, traced=False):
        buf = ctypes.create_string_buffer(lib.lga_e3_args_bytes())
        IA = ctypes.c_int * 5
        lib.lga_e3_fill_args(buf, ctypes.c_void_p(layers_dev.data_ptr()), L, C, Hr, Gr, Ir, Kp, S, esplits, gq, gp, gi,
                             IA(*ru), IA(*units), Nq, ctypes.c_void_p(p.data_ptr()), ctypes.c_void_p(x0.data_ptr()),
                             ctypes.c_void_p(act.data_ptr()), ctypes.c_longlong(stride), IA(*offs),
                             ctypes.c_void_p(ews.data_ptr()), ctypes.c_void_p(ctr.data_ptr()),
                             ctypes.c_void_p(err.data_ptr()), ctypes.c_float(1e-5), ctypes.c_float(scale), compute,
                             ctypes.c_void_p(trace.data_ptr() if traced else 0))
        return torch.frombuffer(bytearray(buf.raw), dtype=torch.uint8).to(dev)  # the kernel reads Args from HBM

    # compute bit 0: consumers compute; bit 1: static unit ranges (no claim atomics); 4 + bits: the same, traced
    bufs = {m: make_args(m) for m in (0, 1, 2, 3)}
    bufs[7] = make_args(3, traced=True)
    bufs[5] = make_args(1, traced=True)
    bufs[6] = make_args(2, traced=True)

    def f_engine(compute=1):
        def run():
            ctr.zero_()
            rc = lib.lga_e3_launch(ctypes.c_void_p(bufs[compute].data_ptr()), n_cu,
                                   ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            assert rc == 0, rc
        return run

    if args.check:
        for m in (1, 3):
            print(f"-- check, {'static ranges' if m & 2 else 'dynamic claims'}", flush=True)
            try:
                check(f_engine(m), W, x0, act, offs, stride, Nq, Kp, C, Ir, Hr, Gr, hs, pos, scale, err, ews, L)
            except AssertionError as e:
                print(f"check FAILED at {e}", flush=True)
    if args.trace:
        for m, name in ((7, "static ranges"), (6, "static ranges, consumers computing nothing (floor)"),
                        (5, "dynamic claims")):
            for _ in range(3):  # warm
                f_engine(m)()
            torch.cuda.synchronize()
            trace.zero_()
            f_engine(m)()
            torch.cuda.synchronize()
            if int(err[0].item()) != 0:
                dump(err)
            show_trace(trace.cpu().numpy(), L, n_cu, name, ncons)
    t = {}
    for r in range(3):
        t.setdefault("per-op", []).append(time_graph(f_layer, L))
        t.setdefault("engine", []).append(time_graph(f_engine(1), L))
        t.setdefault("engine static", []).append(time_graph(f_engine(3), L))
        if args.floor:
            t.setdefault("engine floor", []).append(time_graph(f_engine(0), L))
            t.setdefault("static floor", []).append(time_graph(f_engine(2), L))
        torch.cuda.synchronize()
        if int(err[0].item()) != 0:
            dump(err)
    for k, v in t.items():
        print(f"{args.geom} {k:14s} " + " ".join(f"{x:6.2f}" for x in v) + f"  us/layer (best {min(v):.2f})",
              flush=True)
    print(f"{args.geom} engine / per-op = {min(t['engine']) / min(t['per-op']):.3f}, "
          f"static {min(t['engine static']) / min(t['per-op']):.3f}", flush=True)


def show_trace(tr, L, n_cu, name, ncons):
    """Per op of the middle layers, times (us) relative to the op's edge E = the last consumer end of the previous
    op on any CU: median / max over CUs of each event, and the op's span E(op + 1) - E(op)."""
    ev = tr[256:].reshape(5 * L, n_cu, 32).astype(np.float64) / 100.0  # 100 MHz -> us
    t0 = tr[:n_cu].astype(np.float64).min() / 100.0
    S0, E0 = 6, 6 + ncons
    ends = np.where(ev[:, :, E0:E0 + ncons] > 0, ev[:, :, E0:E0 + ncons], 0).max(axis=2)  # [op][cu] last end
    E = ends.max(axis=1)  # op complete (approx.: last consumer end)
    kinds = "QAPFD"
    print(f"trace ({name}): launch span {E[-1] - t0:.1f} us for {L} layers; per op of layers {L // 2 - 1}-{L // 2}, "
          f"us relative to the previous op's completion (median / max over CUs; '-' no CU recorded it)", flush=True)
    cols = ["claim0", "claim1", "load0", "load1", "edge", "staged", "start", "end"]
    print("op      span  " + "  ".join(f"{c:>13s}" for c in cols), flush=True)
    for op in range(5 * (L // 2 - 1), 5 * (L // 2 + 1)):
        Eprev = E[op - 1]
        starts = np.where(ev[op, :, S0:E0] > 0, ev[op, :, S0:E0], np.inf).min(axis=1)
        vals = [ev[op, :, 0], ev[op, :, 1], ev[op, :, 2], ev[op, :, 3], ev[op, :, 4], ev[op, :, 5], starts, ends[op]]
        cells = []
        for v in vals:
            v = v[(v > 0) & np.isfinite(v)]
            cells.append("-" if v.size == 0 else f"{np.median(v) - Eprev:6.2f}/{v.max() - Eprev:6.2f}")
        print(f"{op // 5:2d}{kinds[op % 5]}  {E[op] - Eprev:7.2f}  " + "  ".join(f"{c:>13s}" for c in cells), flush=True)


def dump(err):
    """Print the engine's timeout records (engine3.hip dbg) and stop."""
    e = err.cpu().numpy().astype("int64")
    recs = e[64:].reshape(256, 8, 128)
    names = {1: "claimer queue", 2: "loader queue", 4: "loader FREE", 8: "wait_done", 16: "staged", 32: "wait_full",
             64: "desc"}
    shown = 0
    from collections import Counter
    print(f"engine error bits {int(e[0]):#x}; timeouts by kind:",
          dict(Counter(names.get(int(c), c) for c in recs[:, :, 0].ravel() if c)), flush=True)
    for cu in range(256):
        for w in range(8):
            r = recs[cu, w]
            if r[0] and shown < 12:
                shown += 1
                print(f"cu {cu} wave {w} {names.get(int(r[0]), r[0])}: ctx {r[1]} {r[2]} {r[3]} | staged {r[4]} "
                      f"gather {r[5]} edge {r[6]} desc_seq {r[7]} cq {r[8]}/{r[9]} gathering {r[10]} | "
                      f"full {r[12:20].tolist()} freed {r[20:28].tolist()} acc_w {[hex(x) for x in r[28:36]]} "
                      f"acc_n {r[36:44].tolist()}", flush=True)
    # per-op accounting across CUs (any wave's snapshot of the CU): claimed units, finished units, closed or not
    for slot in range(8):
        n_sum = fin = closed = incons = 0
        for cu in range(256):
            r = next((recs[cu, w] for w in range(8) if recs[cu, w, 0]), None)
            if r is None:
                continue
            w_, n_ = int(r[28 + slot]), int(r[36 + slot])
            n_sum += n_
            fin += w_ & 0xFFFFFF
            closed += bool(w_ & 0x1000000)
            incons += bool(w_ & 0x1000000) and (w_ & 0xFFFFFF) != n_
        print(f"acc slot {slot}: claimed {n_sum}, finished {fin}, closed on {closed} CUs, count != claimed on {incons}",
              flush=True)
        if incons and slot == 7:
            shown = 0
            for cu in range(256):
                r = next((recs[cu, w] for w in range(8) if recs[cu, w, 0]), None)
                if r is None or not (int(r[28 + slot]) & 0x1000000) or (int(r[28 + slot]) & 0xFFFFFF) == int(r[36 + slot]):
                    continue
                if shown < 4:
                    shown += 1
                    ds = int(r[7])
                    print(f"  cu {cu}: desc_seq {ds}, consumers at descs {r[44:47].tolist()}; ring (desc: op/unit) " +
                          " ".join(f"{d}:{int(r[48 + d % 32])}/{int(r[80 + d % 32])}" for d in range(max(0, ds - 32), ds)),
                          flush=True)
                    for w in range(8):
                        rw = recs[cu, w]
                        if rw[0]:
                            print(f"    wave {w} {names.get(int(rw[0]), rw[0])} ctx {rw[1]} {rw[2]} {rw[3]}", flush=True)
    raise SystemExit(1)


def check(run, W, x0, act, offs, stride, Nq, Kp, C, Ir, Hr, Gr, hs, pos, scale, err, ews, L_):
    """Layer 0 of the engine against references of the same math."""
    w = W[0]
    kc0, vc0 = w["kc"].clone(), w["vc"].clone()
    try:
        _check(run, w, kc0, vc0, x0, act, offs, stride, Nq, Kp, C, Ir, Hr, Gr, hs, pos, scale, err, ews, L_)
    finally:
        w["kc"].copy_(kc0)
        w["vc"].copy_(vc0)


def _check(run, w, kc0, vc0, x0, act, offs, stride, Nq, Kp, C, Ir, Hr, Gr, hs, pos, scale, err, ews, L_):
    failed = []
    run()
    torch.cuda.synchronize()
    if int(err[0].item()) != 0:
        dump(err)
    a = act[:stride]
    e_qkv, e_y, e_xp, e_g, e_xo = (a[offs[i]:offs[i] + n] for i, n in enumerate((Nq, Kp, C, Ir, C)))

    def rel(got, want, name, tol):
        d = (got.float() - want.float()).abs().max().item() / max(want.float().abs().max().item(), 1e-6)
        print(f"check {name:5s}: max rel err {d:.2e}" + ("" if d <= tol else "  FAILED"), flush=True)
        if d > tol:
            failed.append(name)

    r_qkv = ops.q4_gemv(x0, *w["qkv"][:2], Nq, C, w["qkv"][2], 0, norm_weight=w["n1"])
    rel(e_qkv, r_qkv, "qkv", 2e-2)
    # attention over the un-rotated cache with the new row appended at pos (the engine's own qkv row)
    qpk = Hr // Gr
    t = e_qkv.view(Gr, qpk + 2, hs).float()
    kc, vc = kc0.float(), vc0.float()
    kc[:, pos], vc[:, pos] = t[:, qpk], t[:, qpk + 1]
    assert torch.equal(w["kc"][:, pos].float(), t[:, qpk]), "engine did not append k"
    yr = torch.empty(Hr, hs, device=act.device)
    for h in range(Hr):
        gi = h // qpk
        s = kc[gi, :pos + 1] @ t[gi, h % qpk] * scale
        yr[h] = torch.softmax(s, 0) @ vc[gi, :pos + 1]
    d = (e_y.float().view(Hr, hs) - yr).abs().amax(1) / yr.abs().amax(1).clamp_min(1e-6)
    ratio = e_y.float().view(Hr, hs).norm(dim=1) / yr.norm(dim=1)
    print(f"attn per head rel err {[round(x, 3) for x in d.tolist()[:8]]} ... norm ratio "
          f"{[round(x, 3) for x in ratio.tolist()[:8]]}", flush=True)
    # which wrong computation does the engine's y match? (diagnostics for a failing attention check)
    if (e_y.float().view(Hr, hs) - yr).abs().max() > 2e-2 * yr.abs().max():
        ey = e_y.float().view(Hr, hs)

        def variant(fn):
            out = torch.empty(Hr, hs, device=act.device)
            for h in range(Hr):
                out[h] = fn(h // qpk, t[h // qpk, h % qpk])
            return ((ey - out).abs().amax(1) / out.abs().amax(1).clamp_min(1e-6)).median().item()
        n = pos + 1
        cand = {
            "V rows shifted +1": lambda gi, q: torch.softmax(kc[gi, :n] @ q * scale, 0)[:-1] @ vc[gi, 1:n],
            "V rows shifted -1": lambda gi, q: torch.softmax(kc[gi, :n] @ q * scale, 0)[1:] @ vc[gi, :n - 1],
            "no new key": lambda gi, q: torch.softmax(kc[gi, :pos] @ q * scale, 0) @ vc[gi, :pos],
            "scale 1": lambda gi, q: torch.softmax(kc[gi, :n] @ q, 0) @ vc[gi, :n],
            "uniform": lambda gi, q: vc[gi, :n].mean(0),
            "scale x2": lambda gi, q: torch.softmax(kc[gi, :n] @ q * scale * 2, 0) @ vc[gi, :n],
            "scale /2": lambda gi, q: torch.softmax(kc[gi, :n] @ q * scale / 2, 0) @ vc[gi, :n],
            "K of group g+1": lambda gi, q: torch.softmax(kc[(gi + 1) % Gr, :n] @ q * scale, 0) @ vc[gi, :n],
            "V of group g+1": lambda gi, q: torch.softmax(kc[gi, :n] @ q * scale, 0) @ vc[(gi + 1) % Gr, :n],
            "q dims 0-63 only": lambda gi, q: torch.softmax(kc[gi, :n, :64] @ q[:64] * scale, 0) @ vc[gi, :n],
            "q dims 64-127 only": lambda gi, q: torch.softmax(kc[gi, :n, 64:] @ q[64:] * scale, 0) @ vc[gi, :n],
            "q dims 0-63 twice": lambda gi, q: torch.softmax(kc[gi, :n, :64] @ q[:64] * 2 * scale, 0) @ vc[gi, :n],
            "q of group g+1": lambda gi, q: torch.softmax(kc[gi, :n] @ t[(gi + 1) % Gr, 0] * scale, 0) @ vc[gi, :n],
            "k row as q": lambda gi, q: torch.softmax(kc[gi, :n] @ t[gi, qpk] * scale, 0) @ vc[gi, :n],
            "q halves swapped": lambda gi, q: torch.softmax(kc[gi, :n] @ torch.cat([q[64:], q[:64]]) * scale, 0)
            @ vc[gi, :n],
            "q pairs swapped": lambda gi, q: torch.softmax(kc[gi, :n] @ q.view(-1, 2).flip(1).reshape(-1) * scale, 0)
            @ vc[gi, :n],
        }
        for k, fn in cand.items():
            print(f"  attn vs '{k}': median per-head rel err {variant(fn):.3f}", flush=True)
        print(f"  reference per-head rel err median {d.median().item():.3f}", flush=True)
        dump_path = os.environ.get("E3_ATTN_DUMP")
        if dump_path:  # the first two groups' inputs and the engine's outputs, for offline analysis
            nsp_ = ews.numel() // (L_ * Hr * (hs + 4))
            np.savez(dump_path, q=t[:2].cpu().numpy(), kc=kc[:2, :pos + 1].cpu().numpy(),
                     vc=vc[:2, :pos + 1].cpu().numpy(), y=ey[:2].cpu().numpy(),
                     part=ews[:2 * nsp_ * (hs + 4)].view(2, nsp_, hs + 4).cpu().numpy(),
                     scale=np.float32(scale), pos=np.int64(pos))
            print(f"  dumped {dump_path}", flush=True)
        # per split: the engine's published (m, l, o) of layer 0 against the split's own attention
        nsp = ews.numel() // (L_ * Hr * (hs + 4))
        part = ews[:Hr * nsp * (hs + 4)].view(Hr, nsp, hs + 4)
        L1 = pos + 1
        chunk = -(-L1 // nsp)
        l2e = 1.4426950408889634
        for h in range(min(Hr, 2)):
            gi = h // qpk
            for sp in range(nsp):
                lo, hi = min(sp * chunk, L1), min(sp * chunk + chunk, L1)
                if hi <= lo:
                    continue
                sc = (kc[gi, lo:hi] @ t[gi, h % qpk]) * scale * l2e
                m_r = sc.max()
                e_r = torch.exp2(sc - m_r)
                l_r, o_r = e_r.sum(), e_r @ vc[gi, lo:hi]
                m_e, l_e, o_e = part[h, sp, 0], part[h, sp, 1], part[h, sp, 4:]
                print(f"  head {h} split {sp} keys [{lo},{hi}): m {m_e.item():.4f}/{m_r.item():.4f} "
                      f"l {l_e.item():.3f}/{l_r.item():.3f} o rel err "
                      f"{((o_e - o_r).abs().max() / o_r.abs().max()).item():.3f}", flush=True)
    rel(e_y, yr.view(-1), "attn", 2e-2)
    r_xp = ops.q4_gemv(e_y.contiguous(), *w["proj"][:2], C, Kp, w["proj"][2], 0, residual=x0)
    rel(e_xp, r_xp, "proj", 2e-2)
    r_g = ops.q4_gemv_swiglu(e_xp.contiguous(), *w["fc1"][:2], *w["fc2"][:2], Ir, C, w["fc1"][2], 0,
                             norm_weight=w["n2"])
    rel(e_g, r_g, "fc", 3e-2)
    r_xo = ops.q4_gemv(e_g.contiguous(), *w["down"][:2], C, Ir, w["down"][2], 0, residual=e_xp.contiguous())
    rel(e_xo, r_xo, "down", 2e-2)
    assert not failed, failed


if __name__ == "__main__":
    main()
