"""The RCCL ("nccl" backend) branches of the data-parallel path on the GPU box's one card: a world-size-1 process group
over RCCL (the pool has one GPU per box; the driver's 8-GPU scaling run is the N > 1 measurement). What runs here that
the gloo rehearsals do not: the RCCL communicator itself, the weight broadcast of a flat DEVICE tensor in the bf16 wire
format (two collectives plus the PFM_FAST_XW bits) with pfm_set_weight_device loading, and AutoModel's data-parallel
collectives: the input-count agreement, the token-matrix gather (all_gather_into_tensor on device memory) and the
object gather. The case runs in a spawned process, so the pytest process never holds a process group.
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rccl_worker(port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        from funasr_amd.config import paraformer_tiny
        from funasr_amd.distributed import broadcast_state_dict
        from funasr_amd.runtime import PfmEngine
        from funasr_amd.weights import make_weights, param_layout
        from tests.golden.inputs import fbank_input
        out = {"backend": dist.get_backend()}
        cfg = paraformer_tiny()
        sd = make_weights(cfg, seed=3)
        dev = torch.device("cuda", 0)
        flat, xw = broadcast_state_dict(param_layout(cfg), sd, device=dev, keep_on_device=True, wire="bf16",
                                        with_xw=True)
        out["flat_device"] = str(flat.device)
        e_wire = PfmEngine(cfg, 0)
        e_wire.load_flat_device(flat, param_layout(cfg), fast_only=True, wire_xw=xw)
        e_host = PfmEngine(cfg, 0)
        e_host.load_state_dict(sd)
        x, l = fbank_input(seed=5, B=6, T=90, lens=[90, 77, 64, 90, 33, 81], dim=cfg.input_size)
        xs, ls = torch.from_numpy(x).to(dev), torch.from_numpy(l).to(dev)
        rw = e_wire.run(xs, ls, mode="fast")
        rh = e_host.run(xs, ls, mode="fast")
        torch.cuda.synchronize()
        out["wire_equal"] = bool(torch.equal(rw["ntok"].cpu(), rh["ntok"].cpu()) and
                                 torch.equal(rw["tokens"].cpu(), rh["tokens"].cpu()))
        # the data-parallel gathers over RCCL: input-count agreement, the token-matrix block (all_gather_into_tensor
        # of device memory) and the object gather of the non-greedy result kinds
        from funasr_amd.distributed import agree_item_count, gather_results, gather_token_matrices
        out["count"] = agree_item_count(6)
        r1 = e_host.run(xs[:4], ls[:4], mode="fast")
        r2 = e_host.run(xs[4:], ls[4:], mode="fast")
        toks, ntok, index = gather_token_matrices([(r1["tokens"], r1["ntok"]), (r2["tokens"], r2["ntok"])],
                                                  [3, 1, 0, 5, 2, 4])
        out["gathered"] = (toks.tolist(), ntok.tolist(), index.tolist())
        out["local"] = ([t for r in (r1, r2) for t in r["tokens"].cpu().tolist()],
                        [n for r in (r1, r2) for n in r["ntok"].cpu().tolist()])
        out["objects"] = gather_results([(0, "a"), (1, {"k": [1, 2]})])
        q.put(out)
    except Exception as ex:  # noqa: BLE001
        import traceback
        q.put({"error": f"{ex!r}\n{traceback.format_exc()}"})
    finally:
        dist.destroy_process_group()


def test_rccl_world1_broadcast_and_gather():
    """World size 1 over RCCL: the bf16-wire device broadcast decodes bit-identically to the host-loaded engine; the
    input-count agreement, the token-matrix gather (device tensors, rows with their input indices) and the object
    gather return this rank's data unchanged."""
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    out = q.get(timeout=240)
    p.join(timeout=60)
    assert "error" not in out, out.get("error")
    assert p.exitcode == 0
    assert out["backend"] == "nccl"
    assert out["flat_device"].startswith("cuda")
    assert out["wire_equal"]
    assert out["count"] == 6
    toks, ntok, index = out["gathered"]
    lt, ln = out["local"]
    assert index == [3, 1, 0, 5, 2, 4]
    assert ntok == ln and sum(ln) > 0
    for r in range(6):   # rows padded to the widest part with -1; each row's tokens are its batch's decode
        assert toks[r][:ln[r]] == lt[r][:ln[r]], r
    assert out["objects"] == [(0, "a"), (1, {"k": [1, 2]})]
