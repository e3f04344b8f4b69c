from .transformer import DominoLlamaDecoderLayer, apply_domino  # noqa: F401
