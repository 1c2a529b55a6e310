"""Worker for tests/test_gpu_tp.py::test_tp_matches_reference_tp_fixture (torch.distributed.run, all ranks on cuda:0,
gloo group + the xGMI all-reduce). Builds the tiny configs of tests/golden/make_golden_tp.py from the same
``oracle.synth`` weights with the PRODUCT's generate/tp.py ``tensor_parallel``, quantizes every float shard on the
device (int4-g128, group fitted per shard) or keeps bf16, and runs the fixture's prompt + its reference-greedy
tokens teacher-forced; rank 0 writes the logits."""

import os
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO / "lit-gpt_amd"), str(REPO), str(REPO / "tests" / "golden")]

from generate import tp as gtp  # noqa: E402
from lit_gpt import GPT, Config, comm  # noqa: E402
from lit_gpt.quantize import QuantizedPrecision  # noqa: E402
from oracle import synth  # noqa: E402
from tp_geometry_worker import router_gap_hooks  # noqa: E402

DEV = torch.device("cuda", 0)


@torch.inference_mode()
def main():
    out, fam, mode = sys.argv[1], sys.argv[2], sys.argv[3]
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    comm.set_default(comm.XgmiAllReduce(device=DEV))
    from make_golden_tp import FAMILIES, STEPS, T

    name, kw = FAMILIES[fam]
    cfg = Config.from_name(name, **kw)
    sd = synth.state_dict(cfg, seed=17)
    g = np.load(REPO / "tests" / "golden" / "g4_tp_logits.npz")
    key = f"{fam}_w{world}_{'q4g' if mode != 'bf16' else 'fp32'}_bfloat16"
    toks = g[f"{key}_tokens"]
    prompt = torch.from_numpy(g[f"{fam}_prompt"]).to(DEV)
    model = GPT(cfg)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    gtp.tensor_parallel(gtp.Fabric(world, rank), model)
    if mode != "bf16":  # quantize the float shards (the fixture quantized them in fp32 too)
        QuantizedPrecision(mode).convert_module(model, DEV)
    model = model.to(device=DEV, dtype=torch.bfloat16)
    model.max_seq_length = T + STEPS + 1
    model.set_kv_cache(1, device=DEV)
    gaps, step_gaps = [], []
    router_gap_hooks(model, gaps)

    def record(lg):
        step_gaps.append(min(gaps, default=float("inf")))
        gaps.clear()
        return lg[0, -1].float()

    logits = [record(model(prompt.view(1, -1), torch.arange(T, device=DEV), last_token_only=True))]
    for s in range(STEPS):
        logits.append(record(model(torch.tensor([[int(toks[s])]], device=DEV), torch.tensor([T + s], device=DEV),
                                   last_token_only=True)))
    err = comm.get_default().errors()
    if rank == 0:
        np.savez(out, logits=torch.stack(logits).cpu().numpy(), ref=g[f"{key}_logits"],
                 ref_f32=g[f"{key}_logits_f32"], gaps=np.array(step_gaps), comm_err=err)
    dist.barrier()
    comm.get_default().close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
