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
import ctypes
import math
import sys
from pathlib import Path

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
    lib = ctypes.CDLL(str(REPO / "tools" / "_ab" / "liblga_engine3.so"))
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
    units = [-(-Nq // ru[0]), Gr * splits, -(-C // ru[2]), -(-Ir // ru[3]), -(-C // ru[4])]
    offs = [0]
    for n in (Nq, Kp, C, Ir):
        offs.append(offs[-1] + ((n + 63) // 64) * 64)
    stride = offs[-1] + ((C + 63) // 64) * 64
    act = torch.zeros(L * stride, device=dev, dtype=torch.bfloat16)
    ews = torch.zeros(L * Hr * splits * (hs + 4), device=dev, dtype=torch.float32)
    ctr = torch.zeros(lib.lga_e3_counter_words(L, Gr), device=dev, dtype=torch.int32)
    err = torch.zeros(64 + 256 * 8 * 128, device=dev, dtype=torch.int32)  # word 0: error bits; then per-wave records
    n_cu = ops.num_cus()
    assert Hr == Gr, "the lab engine covers one query head per group"
    print(f"{args.geom}: rank H={Hr} G={Gr} I={Ir} Kp={Kp} splits={splits} rows/unit {ru} units {units} "
          f"LDS {lib.lga_e3_lds_bytes()} B, {n_cu} CUs", flush=True)

    def make_args(compute):
        buf = ctypes.create_string_buffer(lib.lga_e3_args_bytes())
        IA = ctypes.c_int * 5
        lib.lga_e3_fill_args(buf, ctypes.c_void_p(layers_dev.data_ptr()), L, C, Hr, Gr, Ir, Kp, S, splits, gq, gp, gi,
                             IA(*ru), IA(*units), Nq, ctypes.c_void_p(p.data_ptr()), ctypes.c_void_p(x0.data_ptr()),
                             ctypes.c_void_p(act.data_ptr()), ctypes.c_longlong(stride), IA(*offs),
                             ctypes.c_void_p(ews.data_ptr()), ctypes.c_void_p(ctr.data_ptr()),
                             ctypes.c_void_p(err.data_ptr()), ctypes.c_float(1e-5), ctypes.c_float(scale), compute)
        return torch.frombuffer(bytearray(buf.raw), dtype=torch.uint8).to(dev)  # the kernel reads Args from HBM

    bufs = {1: make_args(1), 0: make_args(0)}

    def f_engine(compute=1):
        def run():
            ctr.zero_()
            rc = lib.lga_e3_launch(ctypes.c_void_p(bufs[compute].data_ptr()), n_cu,
                                   ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            assert rc == 0, rc
        return run

    if args.check:
        check(f_engine(1), W, x0, act, offs, stride, Nq, Kp, C, Ir, Hr, Gr, hs, pos, scale, err)
    t = {}
    for r in range(3):
        t.setdefault("per-op", []).append(time_graph(f_layer, L))
        t.setdefault("engine", []).append(time_graph(f_engine(1), L))
        if args.floor:
            t.setdefault("engine floor", []).append(time_graph(f_engine(0), L))
        torch.cuda.synchronize()
        if int(err[0].item()) != 0:
            dump(err)
    for k, v in t.items():
        print(f"{args.geom} {k:14s} " + " ".join(f"{x:6.2f}" for x in v) + f"  us/layer (best {min(v):.2f})",
              flush=True)
    print(f"{args.geom} engine / per-op = {min(t['engine']) / min(t['per-op']):.3f}", flush=True)


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


def check(run, W, x0, act, offs, stride, Nq, Kp, C, Ir, Hr, Gr, hs, pos, scale, err):
    """Layer 0 of the engine against references of the same math."""
    w = W[0]
    kc0, vc0 = w["kc"].clone(), w["vc"].clone()
    run()
    torch.cuda.synchronize()
    if int(err[0].item()) != 0:
        dump(err)
    a = act[:stride]
    e_qkv, e_y, e_xp, e_g, e_xo = (a[offs[i]:offs[i] + n] for i, n in enumerate((Nq, Kp, C, Ir, C)))

    def rel(got, want, name, tol):
        d = (got.float() - want.float()).abs().max().item() / max(want.float().abs().max().item(), 1e-6)
        print(f"check {name:5s}: max rel err {d:.2e}", flush=True)
        assert d <= tol, name

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
    rel(e_y, yr.view(-1), "attn", 2e-2)
    r_xp = ops.q4_gemv(e_y.contiguous(), *w["proj"][:2], C, Kp, w["proj"][2], 0, residual=x0)
    rel(e_xp, r_xp, "proj", 2e-2)
    r_g = ops.q4_gemv_swiglu(e_xp.contiguous(), *w["fc1"][:2], *w["fc2"][:2], Ir, C, w["fc1"][2], 0,
                             norm_weight=w["n2"])
    rel(e_g, r_g, "fc", 3e-2)
    r_xo = ops.q4_gemv(e_g.contiguous(), *w["down"][:2], C, Ir, w["down"][2], 0, residual=e_xp.contiguous())
    rel(e_xo, r_xo, "down", 2e-2)
    w["kc"].copy_(kc0)
    w["vc"].copy_(vc0)


if __name__ == "__main__":
    main()
