"""Long-context RoPE fixture from the REFERENCE's own build_rope_cache (lit_gpt/model.py:746-764).

Run once here (never on the GPU box; /root/reference does not exist there):
    python tests/golden/make_golden_rope.py
Writes g5_rope_long.npz: cos / sin rows of a 32768-row, 128-element cache around the bf16 position-rounding
boundaries (4095-4200, 8185-8200, 16380-16400, 32760-32767) at base 1e4 (Llama-2) and 1e6 (Mixtral,
lit_gpt/config.py:1304), built under an fp32 default dtype and under a bf16 one (the reference's init_tensor context
at bf16-true precision, where the position range is rounded to bf16 before the outer product, model.py:758-759).
The reference is imported with make_golden.import_reference (stand-ins for Lightning only).
"""

from __future__ import annotations

import numpy as np
import torch

from make_golden import HERE, import_reference

ROWS = np.r_[4095:4201, 8185:8201, 16380:16401, 32760:32768]


def main():
    _, model_mod, _, _ = import_reference()
    out = {"rows": ROWS.astype(np.int64)}
    for base in (10000, 1000000):
        for dt, tag in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
            prev = torch.get_default_dtype()
            torch.set_default_dtype(dt)
            try:
                cos, sin = model_mod.build_rope_cache(32768, 128, base=base)
            finally:
                torch.set_default_dtype(prev)
            out[f"cos_{base}_{tag}"] = cos[ROWS].float().numpy()
            out[f"sin_{base}_{tag}"] = sin[ROWS].float().numpy()
            print(base, tag, cos.dtype, float(cos[ROWS].double().sum()))
    np.savez_compressed(HERE / "g5_rope_long.npz", **out)


if __name__ == "__main__":
    main()
