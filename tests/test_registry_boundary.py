"""The plugin route into the reference's own registry, checked against the reference code itself (build
container only: /root/reference is absent on the GPU box, where this test skips). No GPU, no inference.

In a child process (so the stubbed `funasr` package does not leak into other tests) the reference is imported
as tests/golden/make_golden.py does (kaldiio / librosa / torchaudio / omegaconf stubbed,
funasr/__init__.py bypassed), then:
  * funasr_amd.register.install_into_funasr() re-registers the HIP classes into the reference's
    `funasr.register.tables` (funasr/register.py:60-65 allows re-registration of a key);
  * the class the reference's AutoModel.build_model would resolve (funasr/auto/auto_model.py:260-288:
    tables.model_classes.get(kwargs["model"]), then model_class(**conf, vocab_size=...)) is the HIP class;
  * the reference's own load_pretrained_model (funasr/train_utils/load_pretrained_model.py:14-104, the
    init_param route of build_model) loads a torch.save'd {"state_dict": ...} into it with strict=True, and
    the weights read back equal the saved ones bit for bit.
"""
import os
import subprocess
import sys
import textwrap

import pytest

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent(r"""
    import sys, os
    sys.path.insert(0, ROOT)
    sys.dont_write_bytecode = True
    import numpy as np, torch
    from tests.golden import make_golden   # imports the reference under the stubs (funasr = REF/funasr)
    from funasr.register import tables as ref_tables
    from funasr.train_utils.load_pretrained_model import load_pretrained_model
    import funasr_amd
    from funasr_amd.register import install_into_funasr
    from funasr_amd.config import paraformer_tiny
    from funasr_amd.weights import make_weights

    ref_para = ref_tables.model_classes["Paraformer"]
    assert ref_para.__module__.startswith("funasr.models"), ref_para
    assert install_into_funasr() is True   # imports and registers every HIP model class
    cls = ref_tables.model_classes.get("Paraformer")
    assert cls is funasr_amd.Paraformer, cls
    for k in ("SenseVoiceSmall", "CTTransformer", "FsmnVADStreaming", "ParaformerStreaming"):
        assert ref_tables.model_classes[k] is funasr_amd.register.tables.model_classes[k], k

    cfg = paraformer_tiny()
    kw = cfg.reference_kwargs()
    vocab = kw.pop("vocab_size")
    model = cls(**kw, vocab_size=vocab)           # auto_model.py:281 calling convention
    sd = {k: torch.from_numpy(v) for k, v in make_weights(cfg, seed=3).items()}
    path = os.path.join(TMP, "model.pt")
    torch.save({"state_dict": sd}, path)
    load_pretrained_model(path=path, model=model, ignore_init_mismatch=True, map_location="cpu")
    back = model.state_dict()
    assert set(back) == set(sd), (len(back), len(sd))
    bad = [k for k in sd if not torch.equal(back[k].float(), sd[k].float())]
    assert not bad, bad[:5]
    print("REGISTRY_OK", len(sd))
""")


@pytest.mark.skipif(not os.path.isdir(f"{REF}/funasr"), reason="reference tree not present (GPU box)")
def test_install_into_reference_registry_and_load_pretrained(tmp_path):
    code = f"ROOT = {ROOT!r}\nTMP = {str(tmp_path)!r}\n" + CHILD
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0 and "REGISTRY_OK" in p.stdout, p.stdout[-2000:] + p.stderr[-4000:]
