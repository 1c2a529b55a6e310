"""CPU-side checks of the C-ABI library: it loads without a GPU and exports every symbol include/*.h declares."""

import ctypes
import re
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
HEADER = REPO / "include" / "litgpt_amd.h"


def header_symbols():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(lga_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib_path():
    from lit_gpt import ops

    if not ops.LIB_PATH.is_file():
        subprocess.run(["make", "-C", str(REPO / "lit-gpt_amd" / "csrc"), "-j8"], check=True)
    return ops.LIB_PATH


def test_library_exports_every_header_symbol(lib_path):
    syms = header_symbols()
    assert len(syms) >= 14
    lib = ctypes.CDLL(str(lib_path))
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header(lib_path):
    from lit_gpt import ops

    assert sorted(ops.SIGNATURES) == header_symbols()
    lib = ops.load_library()
    assert lib.lga_version() >= 1
    assert lib.lga_attention_workspace_bytes(1, 32, 128, 36) == 32 * 36 * 132 * 4  # (m, l, 2 pad, o[hs]) fp32


def test_argument_validation_without_gpu(lib_path):
    """Bad shapes are rejected by the C entry points before any launch (no GPU needed)."""
    from lit_gpt import ops

    lib = ops.load_library()
    rc = lib.lga_q4_gemv(None, None, None, None, None, None, 1e-5, None, 1, 1, 1, 0, -1, None)
    assert rc != 0 and b"null" in lib.lga_last_error_string()
    rc = lib.lga_quantize(ctypes.c_void_p(16), 0, ctypes.c_void_p(16), ctypes.c_void_p(16), 4, 100, 128, 0, None)
    assert rc != 0 and b"multiple" in lib.lga_last_error_string()


def test_library_is_gfx950_code_object(lib_path):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", str(lib_path)], capture_output=True,
                         text=True)
    assert ".hip_fatbin" in out.stdout
    blob = Path(lib_path).read_bytes()
    assert b"gfx950" in blob


def test_ops_refuse_cpu_tensors(lib_path):
    import torch

    from lit_gpt import ops

    with pytest.raises(RuntimeError, match="GPU tensor"):
        ops.rmsnorm(torch.zeros(2, 8, dtype=torch.bfloat16), torch.ones(8, dtype=torch.bfloat16), 1e-5)
    with pytest.raises(RuntimeError, match="GPU tensor"):
        ops.argmax(torch.zeros(8, dtype=torch.bfloat16))


def test_missing_library_fails_loudly(tmp_path):
    from lit_gpt import ops

    with pytest.raises(ops.NativeLibraryError, match="no CPU fallback"):
        ops.load_library(tmp_path / "nope.so")


def _kernel_scratch(lib_path):
    """{kernel symbol: (private segment bytes per lane, VGPR spills)} of every gfx950 kernel in the library: the clang offload
    bundles embedded in the .so (one per translation unit), each kernel's `.private_segment_fixed_size` from the code
    object's metadata note (llvm-readelf --notes)."""
    import os
    import struct
    import tempfile

    readelf = Path("/opt/rocm/lib/llvm/bin/llvm-readelf")
    if not readelf.is_file():
        pytest.skip("llvm-readelf not found")
    data = Path(lib_path).read_bytes()
    out, pos = {}, 0
    while (i := data.find(b"__CLANG_OFFLOAD_BUNDLE__", pos)) >= 0:
        n, off = struct.unpack_from("<Q", data, i + 24)[0], i + 32
        for _ in range(n):
            o, sz, ts = struct.unpack_from("<QQQ", data, off)
            triple = data[off + 24:off + 24 + ts].decode()
            off += 24 + ts
            if "gfx950" not in triple or not sz:
                continue
            with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
                f.write(data[i + o:i + o + sz])
            notes = subprocess.run([str(readelf), "--notes", f.name], capture_output=True, text=True).stdout
            os.unlink(f.name)
            for blk in notes.split("  - .")[1:]:
                name = re.search(r"\.name:\s+(\S+)", blk)
                scratch = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk)
                spill = re.search(r"\.vgpr_spill_count:\s+(\d+)", blk)
                if name and scratch:
                    out[name.group(1)] = (int(scratch.group(1)), int(spill.group(1)) if spill else 0)
        pos = i + 1
    return out


def test_decode_kernels_use_no_scratch(lib_path):
    """Round 6 found every decode GEMV kernel spilling its butterfly partials to scratch (a select of two array loads
    folded into one load through a selected pointer: a scratch round trip per butterfly level in each wave's tail).
    Guard: no decode-path kernel (GEMV, streaming GEMV, MoE, attention, all-reduce, sampling) has a private segment
    or spills VGPRs.
    The prefill fallback GEMM (gemm.hip, shapes the fused kernel declines) is the one known exception."""
    scratch = _kernel_scratch(lib_path)
    assert len(scratch) > 100, len(scratch)
    decode = re.compile(r"gemv|attn_kernel|moe_|allreduce|comm|sample|argmax|rope|rmsnorm")
    bad = {k: v for k, v in scratch.items() if (v[0] or v[1]) and decode.search(k)}
    assert not bad, bad
