"""Class registry mirroring funasr/register.py (tables.register(table, key), :7-84).

`tables.model_classes["Paraformer"]` etc. resolve to the HIP-backed classes of this package.
`install_into_funasr()` additionally re-registers them into an importable reference
`funasr.register.tables` (re-registration of an existing key is allowed there, :60-65), which
is the drop-in route for code that builds models through the reference's AutoModel.
"""
from __future__ import annotations

from typing import Callable, Dict


class RegisterTables:
    def __init__(self):
        self.model_classes: Dict[str, type] = {}
        self.frontend_classes: Dict[str, type] = {}
        self.tokenizer_classes: Dict[str, type] = {}

    def register(self, table: str, key: str) -> Callable[[type], type]:
        def deco(cls):
            getattr(self, table)[key] = cls
            return cls
        return deco

    def print(self, key: str = None):
        for name in ("model_classes", "frontend_classes", "tokenizer_classes"):
            if key is None or key in name:
                print(name, sorted(getattr(self, name)))


tables = RegisterTables()


def install_into_funasr() -> bool:
    """Register the HIP classes into the reference's registry if the reference is importable."""
    try:
        from funasr.register import tables as ref_tables  # type: ignore
    except Exception:
        return False
    # the model modules register themselves on import (lazy in funasr_amd/__init__.py)
    from . import model, punc, sense_voice, streaming, vad  # noqa: F401
    for table in ("model_classes", "frontend_classes", "tokenizer_classes"):
        for k, cls in getattr(tables, table).items():
            ref_tables.register(table, k)(cls)
    return True
