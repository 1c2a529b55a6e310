"""Generate golden vectors by running the REFERENCE (/root/reference) on the CPU in this container.

Run once here (never on the GPU box; /root/reference does not exist there):
    python tests/golden/make_golden.py
Outputs small ``.npz`` fixtures next to this script. Weights come from ``oracle.synth`` (counter-based,
regenerable anywhere), so fixtures carry only prompts, token ids and logits.

The reference cannot be imported as-is (lit_gpt/__init__.py:10-17 needs Lightning, lit_gpt/utils.py:12-17
imports it); per SURVEY §8c the package is registered with ``__path__`` pointing at the reference
sources (skipping its ``__init__``), with tiny stand-ins for ``lit_gpt.utils`` and ``lightning``. Only
the reference's own model/generate code runs.
"""

from __future__ import annotations

import sys
import types
from pathlib import Path

import numpy as np
import torch

REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))


def import_reference():
    pkg = types.ModuleType("lit_gpt")
    pkg.__path__ = [str(REF / "lit_gpt")]
    sys.modules["lit_gpt"] = pkg
    utils = types.ModuleType("lit_gpt.utils")

    def find_multiple(n, k):
        assert k > 0
        return n if n % k == 0 else n + k - n % k

    utils.find_multiple = find_multiple
    utils.check_valid_checkpoint_dir = lambda *a, **k: None
    utils.get_default_supported_precision = lambda training: "32-true"
    utils.load_checkpoint = lambda *a, **k: None
    sys.modules["lit_gpt.utils"] = utils
    L = types.ModuleType("lightning")
    L.Fabric = object
    L.seed_everything = lambda s: torch.manual_seed(s)
    fab = types.ModuleType("lightning.fabric")
    plugins = types.ModuleType("lightning.fabric.plugins")
    plugins.BitsandbytesPrecision = object
    futils = types.ModuleType("lightning.fabric.utilities")
    futils.rank_zero_only = lambda f: f
    sys.modules.update({"lightning": L, "lightning.fabric": fab, "lightning.fabric.plugins": plugins,
                        "lightning.fabric.utilities": futils})
    tok = types.ModuleType("lit_gpt.tokenizer")
    tok.Tokenizer = object
    sys.modules["lit_gpt.tokenizer"] = tok
    import lit_gpt.model as model
    import lit_gpt.config as config

    pkg.GPT, pkg.Config, pkg.Tokenizer = model.GPT, config.Config, object
    sys.path.insert(0, str(REF))
    import generate.base as gbase
    import generate.tp as gtp

    return config, model, gbase, gtp


def ref_model(model_mod, cfg, sd, dtype=torch.float32, max_seq=None, default_dtype=None):
    m = model_mod.GPT(cfg)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    m = m.to(dtype).eval()
    if default_dtype is not None:
        prev = torch.get_default_dtype()
        torch.set_default_dtype(default_dtype)
    m.max_seq_length = max_seq or cfg.block_size
    m.set_kv_cache(batch_size=1)
    if default_dtype is not None:
        torch.set_default_dtype(prev)
    return m


@torch.inference_mode()
def run_teacher_forced(m, prompt, steps):
    """Prefill then `steps` greedy decode steps with the reference's own generate loop; also logits per step."""
    logits_all = []
    T = prompt.numel()
    lg = m(prompt.view(1, -1), torch.arange(T))
    logits_all.append(lg[0, -1].float().clone())
    tok = torch.argmax(lg[0, -1]).view(1).to(prompt.dtype)
    toks = [tok]
    for s in range(steps - 1):
        lg = m(tok.view(1, 1), torch.tensor([T + s]))
        logits_all.append(lg[0, -1].float().clone())
        tok = torch.argmax(lg[0, -1]).view(1).to(prompt.dtype)
        toks.append(tok)
    return torch.cat(toks), torch.stack(logits_all)


def main():
    from oracle import quant, synth

    config, model_mod, gbase, gtp = import_reference()
    torch.manual_seed(0)
    out = {}

    # ---- G1: pythia-160m fp32, random init, 16-token prompt, greedy 128 tokens (config 1) ----
    cfg = config.Config.from_name("pythia-160m")
    sd = synth.state_dict(cfg, seed=1234)
    prompt = torch.from_numpy(synth.token_ids(16, cfg.vocab_size, seed=1234))
    m = ref_model(model_mod, cfg, sd, max_seq=16 + 128)
    y = gbase.generate(m, prompt, 16 + 128, temperature=0.0, top_k=None, eos_id=None)
    m.clear_kv_cache()
    m.set_kv_cache(batch_size=1)
    toks, logits = run_teacher_forced(m, prompt, 128)
    assert torch.equal(toks, y[16:]), "generate() and the teacher-forced loop disagree"
    top2 = torch.topk(logits, 2, dim=-1).values
    np.savez_compressed(HERE / "g1_pythia160m_greedy.npz", prompt=prompt.numpy(), tokens=y.numpy(),
                        step0_logits=logits[0].numpy(), margins=(top2[:, 0] - top2[:, 1]).numpy(),
                        logits_sum=logits.sum(-1).numpy(), logits_absmax=logits.abs().max(-1).values.numpy())
    print("G1 done", y[16:26].tolist())

    # ---- G2: tiny Llama-family models, fp32, full logits for prefill + 15 decode steps ----
    tiny = {
        "llama_mha": dict(name="Llama-2-7b-hf", n_layer=2, n_embd=256, n_head=4, intermediate_size=640,
                          vocab_size=1000, padding_multiple=64, block_size=256),
        "llama_gqa": dict(name="Llama-2-70b-hf", n_layer=2, n_embd=256, n_head=4, n_query_groups=2,
                          intermediate_size=512, vocab_size=1000, padding_multiple=64, block_size=256),
        "llama_mqa": dict(name="Llama-2-7b-hf", n_layer=2, n_embd=256, n_head=4, n_query_groups=1,
                          intermediate_size=384, vocab_size=1000, padding_multiple=64, block_size=256),
        "mixtral": dict(name="Mixtral-8x7B-v0.1", n_layer=2, n_embd=256, n_head=4, n_query_groups=2,
                        intermediate_size=384, n_expert=4, n_expert_per_token=2, padded_vocab_size=1024,
                        vocab_size=1024, block_size=256),
    }
    for key, kw in tiny.items():
        name = kw.pop("name")
        cfg = config.Config.from_name(name, **kw)
        sd = synth.state_dict(cfg, seed=7)
        prompt = torch.from_numpy(synth.token_ids(24, cfg.vocab_size, seed=7))
        variants = {"fp32": sd}
        if key == "llama_mha":
            qsd, nsd = {}, {}
            for k, v in sd.items():
                if k.endswith(".weight") and v.ndim == 2 and not k.startswith("transformer.wte"):
                    qsd[k] = quant.dequantize_q4g(*quant.quantize_q4g(v, 128), 128)
                    nsd[k] = quant.dequantize_nf4(*quant.quantize_nf4(v, 64), 64)
                else:
                    qsd[k] = nsd[k] = v
            variants["q4g"] = qsd
            variants["nf4"] = nsd
        for vname, vsd in variants.items():
            m = ref_model(model_mod, cfg, vsd, max_seq=24 + 16)
            toks, logits = run_teacher_forced(m, prompt, 16)
            out[f"{key}_{vname}_tokens"] = toks.numpy()
            out[f"{key}_{vname}_logits"] = logits.numpy()
        out[f"{key}_prompt"] = prompt.numpy()
        # no-cache full forward (input_pos=None, is_causal path) over prompt+generated
        full = torch.cat([prompt, torch.from_numpy(out[f"{key}_fp32_tokens"][:-1])])
        m = ref_model(model_mod, cfg, sd, max_seq=24 + 16)
        with torch.inference_mode():
            out[f"{key}_nocache_logits"] = m(full.view(1, -1))[0].float().numpy()
        # bf16 (bf16-true) variant with exact positions
        m = ref_model(model_mod, cfg, sd, dtype=torch.bfloat16, max_seq=24 + 16)
        toks, logits = run_teacher_forced(m, prompt, 16)
        out[f"{key}_bf16_tokens"] = toks.numpy()
        out[f"{key}_bf16_logits"] = logits.numpy()
        print("G2", key, out[f"{key}_fp32_tokens"][:8].tolist())
    np.savez_compressed(HERE / "g2_tiny_models.npz", **out)

    # ---- G3: per-op vectors ----
    g3 = {}
    for pos_dtype, tag in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
        prev = torch.get_default_dtype()
        torch.set_default_dtype(pos_dtype)
        cos, sin = model_mod.build_rope_cache(2304, 128, base=10000)
        torch.set_default_dtype(prev)
        g3[f"rope_cos_{tag}"] = cos[2040:2050].numpy()
        g3[f"rope_sin_{tag}"] = sin[2040:2050].numpy()
        g3[f"rope_cos_{tag}_sum"] = cos.double().sum().numpy()
    cos, sin = model_mod.build_rope_cache(64, 16, base=1000000, condense_ratio=2)
    g3["rope_small_cos"], g3["rope_small_sin"] = cos.numpy(), sin.numpy()
    x = torch.from_numpy(synth.normal((1, 3, 64, 16), "rope_x", 1, 1.0))
    g3["rope_x"], g3["rope_y"] = x.numpy(), model_mod.apply_rope(x, cos, sin).numpy()
    from lit_gpt.rmsnorm import RMSNorm

    xn = torch.from_numpy(synth.normal((5, 300), "rms_x", 1, 3.0))
    wn = torch.from_numpy(synth.normal((300,), "rms_w", 1, 1.0))
    rn = RMSNorm(300, eps=1e-5)
    rn.weight.data = wn
    g3["rms_x"], g3["rms_w"] = xn.numpy(), wn.numpy()
    g3["rms_y"] = rn(xn).detach().numpy()
    g3["rms_y_bf16"] = rn.to(torch.bfloat16)(xn.to(torch.bfloat16)).float().detach().numpy()
    logits = torch.tensor([[[24, 4, 98, 77, 47], [65, 70, 32, 67, 24], [92, 32, 88, 36, 62]],
                           [[85, 79, 57, 68, 50], [89, 46, 72, 45, 32], [68, 96, 68, 24, 36]]])
    g3["sample_logits"] = logits.numpy()
    g3["sample_t0"] = gbase.sample(logits, temperature=0.0).numpy()
    tl = torch.tensor([[[1.0, 5.0, 5.0, 2.0, 5.0, -1.0]]])
    g3["sample_ties_logits"] = tl.numpy()
    g3["sample_ties_t0"] = gbase.sample(tl, temperature=0.0).numpy()
    g3["sample_ties_t0_k2"] = gbase.sample(tl, temperature=0.0, top_k=2).numpy()
    np.savez_compressed(HERE / "g3_ops.npz", **g3)

    # ---- G4: tensor_parallel_linear shards via the reference function (Mock fabric) ----
    from unittest.mock import Mock

    g4 = {}
    for world in (2, 4, 8):
        for rank in range(world):
            fab = Mock()
            fab.world_size, fab.global_rank = world, rank
            for style in ("colwise", "rowwise"):
                lin = torch.nn.Linear(16, 24, bias=True)
                lin.weight.data = torch.arange(24 * 16, dtype=torch.float32).reshape(24, 16)
                lin.bias.data = torch.arange(24, dtype=torch.float32)
                try:
                    gtp.tensor_parallel_linear(fab, lin, style)
                    g4[f"w{world}_r{rank}_{style}_weight"] = lin.weight.detach().numpy()
                    g4[f"w{world}_r{rank}_{style}_bias"] = lin.bias.detach().numpy()
                except ValueError:
                    g4[f"w{world}_r{rank}_{style}_error"] = np.array(1)
    np.savez_compressed(HERE / "g4_tp.npz", **g4)
    print("done")


if __name__ == "__main__":
    main()
