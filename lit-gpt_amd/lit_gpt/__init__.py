"""MI355X-native decode path behind the lit_gpt API (reference lit_gpt/__init__.py:27)."""

from lit_gpt.config import Config

__all__ = ["GPT", "Config", "Tokenizer"]


def __getattr__(name):
    if name == "GPT":
        from lit_gpt.model import GPT

        return GPT
    if name == "Tokenizer":
        from lit_gpt.tokenizer import Tokenizer

        return Tokenizer
    raise AttributeError(name)
