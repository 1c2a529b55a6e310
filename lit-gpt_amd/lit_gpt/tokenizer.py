"""Tokenizer wrapper (reference lit_gpt/tokenizer.py:10-109): SentencePiece or HF tokenizers, int32 ids.

Off the hot path (the benchmark uses synthetic ids); kept so ``generate/base.py`` works on real checkpoints.
"""

from __future__ import annotations

import json
from pathlib import Path
from typing import Optional, Union

import torch


class Tokenizer:
    def __init__(self, checkpoint_dir: Union[Path, str]) -> None:
        checkpoint_dir = Path(checkpoint_dir)
        if not checkpoint_dir.exists():
            raise NotADirectoryError(f"The checkpoint directory does not exist: {str(checkpoint_dir)}")
        self.bos_id: Optional[int] = None
        self.eos_id: Optional[int] = None
        self.use_bos = False
        cfg = {}
        if (checkpoint_dir / "tokenizer_config.json").is_file():
            cfg = json.loads((checkpoint_dir / "tokenizer_config.json").read_text())
            self.use_bos = bool(cfg.get("add_bos_token", False))
        if (vocab := checkpoint_dir / "tokenizer.model").is_file():
            from sentencepiece import SentencePieceProcessor

            self.processor = SentencePieceProcessor(model_file=str(vocab))
            self.backend = "sentencepiece"
            self.bos_id, self.eos_id = self.processor.bos_id(), self.processor.eos_id()
        elif (vocab := checkpoint_dir / "tokenizer.json").is_file():
            from tokenizers import Tokenizer as HFTokenizer

            self.processor = HFTokenizer.from_file(str(vocab))
            self.backend = "huggingface"

            def tok_id(t):
                if isinstance(t, dict):
                    t = t.get("content")
                return None if t is None else self.processor.token_to_id(t)

            self.bos_id = tok_id(cfg.get("bos_token"))
            self.eos_id = tok_id(cfg.get("eos_token"))
        else:
            raise NotImplementedError(f"no tokenizer.model / tokenizer.json in {checkpoint_dir}")

    @property
    def vocab_size(self) -> int:
        if self.backend == "huggingface":
            return self.processor.get_vocab_size(with_added_tokens=False)
        return self.processor.vocab_size()

    def encode(self, string: str, device: Optional[torch.device] = None, bos: Optional[bool] = None,
               eos: bool = False, max_length: int = -1) -> torch.Tensor:
        ids = (self.processor.encode(string).ids if self.backend == "huggingface"
               else self.processor.encode(string))
        if (bos if bos is not None else self.use_bos) and self.bos_id is not None:
            ids = [self.bos_id] + ids
        if eos and self.eos_id is not None:
            ids = ids + [self.eos_id]
        if max_length > 0:
            ids = ids[:max_length]
        return torch.tensor(ids, dtype=torch.int, device=device)

    def decode(self, tensor: torch.Tensor) -> str:
        tokens = [tensor.item()] if tensor.ndim == 0 else tensor.tolist()
        return self.processor.decode(tokens)
