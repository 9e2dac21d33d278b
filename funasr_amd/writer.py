"""Kaldi-style result directories for `output_dir=` (funasr/utils/datadir_writer.py:6-73).

`DatadirWriter(path)[sub][name][key] = value` appends the line "key value" to path/sub/name, creating the
directories on the first write and flushing every line; a second write of a key warns ("Duplicated"). As in the
reference, a model creates ONE writer the first time inference() sees output_dir (the `hasattr(self, "writer")`
idiom, paraformer/model.py:549-552), so the files of later calls append to those of earlier ones, and the
files stay open until the writer is closed or collected.
"""
from __future__ import annotations

import warnings
from pathlib import Path
from typing import Dict, Optional, Union


class DatadirWriter:
    def __init__(self, p: Union[Path, str]):
        self.path = Path(p)
        self.children: Dict[str, "DatadirWriter"] = {}
        self.fd = None
        self.keys = set()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __getitem__(self, name: str) -> "DatadirWriter":
        if self.fd is not None:
            raise RuntimeError("This writer points out a file")
        if name not in self.children:
            self.children[name] = DatadirWriter(self.path / name)
        return self.children[name]

    def __setitem__(self, key: str, value: str):
        if self.children:
            raise RuntimeError("This writer points out a directory")
        if key in self.keys:
            warnings.warn(f"Duplicated: {key}")
        if self.fd is None:
            self.path.parent.mkdir(parents=True, exist_ok=True)
            self.fd = self.path.open("w", encoding="utf-8")
        self.keys.add(key)
        self.fd.write(f"{key} {value}\n")
        self.fd.flush()

    def close(self):
        prev = None
        for child in self.children.values():
            child.close()
            if prev is not None and prev.keys != child.keys:
                warnings.warn(f"Ids are mismatching between {prev.path} and {child.path}")
            prev = child
        if self.fd is not None:
            self.fd.close()
            self.fd = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 — interpreter shutdown
            pass


def model_writer(model, kwargs) -> Optional[DatadirWriter]:
    """The model's writer when output_dir is given (created once per model, as the reference does), else None."""
    out = kwargs.get("output_dir")
    if out is None:
        return None
    if getattr(model, "writer", None) is None:
        model.writer = DatadirWriter(out)
    return model.writer
