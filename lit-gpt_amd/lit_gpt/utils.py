"""Small helpers on the decode path (subset of /root/reference/lit_gpt/utils.py used by generate/*)."""

from __future__ import annotations

import sys
from pathlib import Path


def find_multiple(n: int, k: int) -> int:
    """Smallest multiple of ``k`` that is >= ``n`` (reference lit_gpt/utils.py:74-78)."""
    assert k > 0
    if n % k == 0:
        return n
    return n + k - (n % k)


def check_valid_checkpoint_dir(checkpoint_dir: Path) -> None:
    """Same required files as the reference (lit_gpt/utils.py:93-124); exits with status 1 otherwise."""
    checkpoint_dir = Path(checkpoint_dir)
    files = {
        "lit_model.pth": (checkpoint_dir / "lit_model.pth").is_file(),
        "lit_config.json": (checkpoint_dir / "lit_config.json").is_file(),
        "tokenizer.json OR tokenizer.model": (checkpoint_dir / "tokenizer.json").is_file()
        or (checkpoint_dir / "tokenizer.model").is_file(),
        "tokenizer_config.json": (checkpoint_dir / "tokenizer_config.json").is_file(),
    }
    if checkpoint_dir.is_dir() and all(files.values()):
        return
    problem = (f" is missing the files: {[f for f, ok in files.items() if not ok]!r}" if checkpoint_dir.is_dir()
               else " is not a checkpoint directory")
    print(f"--checkpoint_dir {str(checkpoint_dir.absolute())!r}{problem}.", file=sys.stderr)
    raise SystemExit(1)


def get_default_supported_precision(training: bool) -> str:
    """bf16 on MI355X (reference lit_gpt/utils.py:334-347 picks bf16 when the device supports it)."""
    return "bf16-mixed" if training else "bf16-true"
