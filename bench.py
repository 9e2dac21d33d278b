#!/usr/bin/env python3
"""bench.py — RTFx of Paraformer-large offline batch inference on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode fast|exact]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One step = one pfm_run (encoder -> CIF -> decoder -> argmax) over this rank's batch of
B=64 utterances x 30 s (T=500 LFR frames) of synthetic N(0,1) fbank already resident in HBM;
weights are the seeded random-init Paraformer-large (220.08M params), RCCL-broadcast from
rank 0 once before timing. Weak scaling: every rank decodes its own 64 utterances, no
collective inside the timed region. value = audio seconds of all ranks / max-over-ranks wall.

The timed region runs K uninstrumented steps (value, ms_per_step); a second pass of K steps records
HIP events around every GEMM / attention launch for the live roofline (events add queue gaps, so
they are kept out of the headline number; its step time is reported as instrumented_ms_per_step).
Extra JSON fields: `roofline` of the dominant kernel (the MFMA GEMM, live HIP-event timing),
`path_roofline` (whole-path algorithmic FLOPs / step time), `cpu_baseline` (the oracle
torch-CPU restatement timed on a bounded sample on this host), `exact_mode` (the token-exact mode on the
same batch: every GEMM and the attention as split-bf16 x6 MFMA at f32 accuracy) and fast-vs-exact token
agreement, `sensevoice` (config C4) and
`streaming` (config C5: 600 ms chunks of Paraformer-large streaming through pfm_stream_step, one stream's
per-chunk latency and 64 concurrent streams' throughput, plus its own torch-CPU oracle baseline).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "RTFx (audio-sec/sec) Paraformer-large offline batch, 1/2/4/8 MI355X"
PEAK_TFLOPS = {"fast": 2500.0, "exact": 157.3}     # MI355X dense bf16 MFMA / f32 MFMA (MICROARCH guide)
HBM_PEAK_GBS = 8000.0
FRAME_SEC = 0.06                                    # 10 ms shift x lfr_n 6 (paraformer/model.py:491-493)


def progress(msg: str) -> None:
    """One progress line on stderr per finished leg (a long default run stays visibly alive)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def path_flops(T: int, L: np.ndarray) -> float:
    """F(T,L) = 333,634,560 T + 102,400 T^2 + 96,866,304 L + 32,768 L T per utterance."""
    L = np.asarray(L, dtype=np.float64)
    return float(np.sum(333634560.0 * T + 102400.0 * T * T + 96866304.0 * L + 32768.0 * L * T))


def sensevoice_flops(Tq: int, V: int = 25055, blocks: int = 70) -> float:
    """SenseVoiceSmall per utterance of Tq = T + 4 frames: per SAN-M layer 6,291,456 Tq + 2,048 Tq^2
    (QKV, out-proj, FFN, QK^T, PV), +147,456 Tq for the 560-wide layer-0 QKV, CTC head 1,024 V Tq."""
    return blocks * (6291456.0 * Tq + 2048.0 * Tq * Tq) + 147456.0 * Tq + 1024.0 * V * Tq


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def stream_leg(args, dev, torch, make_weights) -> dict:
    import dataclasses
    from funasr_amd.config import paraformer_streaming
    from funasr_amd.runtime import PfmEngine, PfmStreams
    cfg = paraformer_streaming()
    C = args.stream_chunks
    res = {"workload": f"Paraformer-large streaming, chunk [0,10,5] (600 ms), look-back 4/1, {C} chunks "
                       f"({C * 0.6:.0f} s) per stream, synthetic LFR+CMVN rows", "dtype": "bf16" if args.mode == "fast"
                       else "f32", "mode": args.mode}
    # greedy (the released model: ctc_weight 0) and, as BASELINE C5 names it, the joint decoder + CTC prefix beam
    # per chunk (a CTC head, decoding_ctc_weight 0.3, pfm_stream_step_beam)
    for leg, lcfg in (("", cfg), ("beam_", dataclasses.replace(cfg, ctc_weight=0.3))):
        eng = PfmEngine(lcfg, dev.index or 0)
        eng.load_state_dict(make_weights(lcfg, args.seed))
        g = torch.Generator(device=dev)
        g.manual_seed(2000)
        bkw = dict(beam=args.beam, ctc_weight=0.3, penalty=0.0, nbest=1)
        for S in (1, args.stream_batch):
            chunks = torch.randn((C, S, 10, cfg.input_size), generator=g, device=dev, dtype=torch.float32)
            st = PfmStreams(eng, S, (0, 10, 5), 4, 1, args.mode)
            ids = list(range(S))

            def one_stream():
                st.reset(ids)
                toks = 0
                lat = []
                for c in range(C):
                    t0 = time.perf_counter()
                    if leg:
                        r = st.step_beam(ids, chunks[c], [10] * S, [c == C - 1] * S, **bkw)
                        n = r["ntok"][:, 0]
                        toks += int(n.clamp(min=0).sum().item())
                    else:
                        r = st.step(ids, chunks[c], [10] * S, [c == C - 1] * S)
                        toks += int(r["ntok"].sum().item())    # the host needs the tokens of every chunk
                    lat.append(time.perf_counter() - t0)
                return toks, lat

            one_stream()   # warmup (workspace growth, first-call setup)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            toks, lat = one_stream()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            key = leg + ("single" if S == 1 else f"streams_{S}")
            res[key] = {"streams": S, "value": round(S * C * 0.6 / dt, 1), "unit": "audio-sec/sec",
                        "chunk_ms_mean": round(float(np.mean(lat)) * 1e3, 3),
                        "chunk_ms_p90": round(float(np.percentile(lat, 90)) * 1e3, 3),
                        "tokens_per_chunk_mean": round(toks / (S * C), 2)}
            progress(f"streaming {key}: {res[key]['chunk_ms_mean']} ms per chunk")
            if leg:
                res[key]["search"] = (f"beam {args.beam}, decoding_ctc_weight 0.3, CTC over each chunk's 15-row "
                                      f"window, nbest 1")
            del st, chunks
        del eng
    if args.cpu_utts > 0:
        # the oracle's streaming restatement (torch-CPU fp32, one stream): chunks until >= 5 s of CPU time (at most
        # the leg's C chunks), so the sample is seconds, not a few chunk latencies
        from oracle.streaming_ref import StreamState, chunk_step
        w = make_weights(cfg, args.seed)
        torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
        ss = StreamState(cfg, (0, 10, 5), 4, 1)
        xs = torch.randn((C, 10, cfg.input_size), generator=torch.Generator().manual_seed(5))
        chunk_step(xs[0], StreamState(cfg, (0, 10, 5), 4, 1), w, cfg, False)   # warmup (allocator, MKL)
        tc = time.perf_counter()
        nc = 0
        while nc < C and (nc < 10 or time.perf_counter() - tc < 5.0):
            chunk_step(xs[nc], ss, w, cfg, nc == C - 1)
            nc += 1
        dtc = time.perf_counter() - tc
        res["cpu_baseline"] = {"value": round(nc * 0.6 / dtc, 2), "unit": "audio-sec/sec",
                               "cores": torch.get_num_threads(), "kind": "port",
                               "sample": f"1 stream x {nc} chunks ({nc * 0.6:.1f} s of audio) through "
                                         f"oracle/streaming_ref.chunk_step (torch-CPU fp32), {dtc:.2f} s on {cpu_model()}"}
    return res


def punc_leg(args, dev, torch, make_weights) -> dict:
    from funasr_amd.config import ct_transformer
    from funasr_amd.runtime import PfmEngine
    cfg = ct_transformer()
    w = make_weights(cfg, args.seed)
    eng = PfmEngine(cfg, dev.index or 0)
    eng.load_state_dict(w)
    B, T = 64, 200
    g = torch.Generator(device=dev)
    g.manual_seed(3000)
    ids = torch.randint(3, cfg.vocab_size, (B, T), generator=g, device=dev, dtype=torch.int32)
    lens = torch.full((B,), T, dtype=torch.int32, device=dev)
    for _ in range(2):
        eng.run_punc(ids, lens, mode=args.mode)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.punc_steps):
        eng.run_punc(ids, lens, mode=args.mode)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.punc_steps
    res = {"workload": f"CT-Transformer punctuation (released dims: 4 x 256-wide SAN-M, 272,727-word embedding), "
                       f"{B} sequences x {T} words per pfm_run_punc", "value": round(B * T / dt, 1),
           "unit": "words/sec", "ms_per_call": round(dt * 1e3, 3), "dtype": "bf16" if args.mode == "fast" else "f32"}
    if args.cpu_utts > 0:
        from oracle.punc_ref import punc_forward
        torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
        x = ids.cpu().numpy()
        punc_forward(x[:2], [T] * 2, w, cfg)   # warmup
        tc = time.perf_counter()
        reps = 0
        while reps < 1 or time.perf_counter() - tc < 3.0:   # the whole B x T batch, repeated for >= 3 s
            punc_forward(x, [T] * B, w, cfg)
            reps += 1
        dtc = time.perf_counter() - tc
        res["cpu_baseline"] = {"value": round(reps * B * T / dtc, 1), "unit": "words/sec",
                               "cores": torch.get_num_threads(), "kind": "port",
                               "sample": f"{reps} x {B} sequences x {T} words through oracle/punc_ref.punc_forward "
                                         f"(torch-CPU fp32), {dtc:.2f} s on {cpu_model()}"}
    del eng
    return res


def long_audio_leg(args, sd, cfg) -> dict:
    """AutoModel(model=Paraformer-large, vad_model=FSMN-VAD, punc_model=CT-Transformer).generate(wav): the
    whole file-transcription pipeline (inference_with_vad) on one synthetic long waveform with quiet gaps."""
    import torch
    from funasr_amd.auto_model import AutoModel
    from funasr_amd.config import ct_transformer, fsmn_vad
    from funasr_amd.weights import make_weights, vad_test_weights
    from tests.golden.inputs import token_list, vad_waveform
    S = args.long_audio_s
    gaps = [(t + 7.0, t + 8.2) for t in range(0, S - 10, 11)]
    wav = vad_waveform(61, float(S), gaps)
    pcfg, vcfg = ct_transformer(), fsmn_vad()
    am = AutoModel(model="Paraformer", model_conf=dict(ctc_weight=0.0, predictor_bias=1), device="cuda",
                   mode=args.mode, tokenizer_conf=dict(token_list=token_list(cfg.vocab_size)),
                   vad_model="FsmnVADStreaming", vad_kwargs=dict(model_conf={}, frontend="WavFrontendOnline",
                                                                  frontend_conf=dict(lfr_m=5, lfr_n=1),
                                                                  **vcfg.reference_kwargs()),
                   punc_model="CTTransformer", punc_kwargs=dict(model_conf={}, tokenizer="CharTokenizer",
                                                                tokenizer_conf=dict(token_list=token_list(
                                                                    pcfg.vocab_size)), **pcfg.reference_kwargs()),
                   batch_size_s=300, **cfg.reference_kwargs())
    am.model.load_state_dict(sd)
    am.vad_model.load_state_dict(vad_test_weights(vcfg, 0))
    am.punc_model.load_state_dict(make_weights(pcfg, args.seed))
    am.generate(input=wav)   # warmup: workspaces, first-call setup
    torch.cuda.synchronize()
    walls = []
    for _ in range(3):   # one 300 s file takes ~60 ms: the median of three runs
        t0 = time.perf_counter()
        res = am.generate(input=wav)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
    dt = sorted(walls)[1]
    t1 = time.perf_counter()
    vres = am.inference(wav, model=am.vad_model, kwargs=dict(am.vad_kwargs))
    torch.cuda.synchronize()
    dv = time.perf_counter() - t1
    return {"workload": f"{S} s synthetic 16 kHz waveform with quiet gaps: FSMN-VAD (synthetic weights tuned to "
                        f"segment it) -> Paraformer-large ({args.mode}) on duration-sorted batches of <= 300 s -> "
                        f"CT-Transformer punctuation (released dims)",
            "value": round(S / dt, 1), "unit": "audio-sec/sec", "wall_s": round(dt, 3),
            "wall_s_runs": [round(w, 4) for w in walls],
            "segments": len(vres[0]["value"]), "vad_only_value": round(S / dv, 1),
            "text_chars": len(res[0]["text"]) if res else 0}


def generate_leg(args, sd, cfg, feats, lens) -> dict:
    """AutoModel.generate(input=fbank, input_len=lens, data_type="fbank") with a tokenizer: what §8(d) times, the
    reference's model.inference inside AutoModel.inference (funasr/auto/auto_model.py:343-348) -- the decode, the
    token-id readback, detokenisation, sentence_postprocess and the result dicts -- on the headline batch."""
    import torch
    from funasr_amd.auto_model import AutoModel
    from tests.golden.inputs import token_list
    am = AutoModel(model="Paraformer", model_conf=dict(ctc_weight=0.0, predictor_bias=1), device="cuda",
                   mode=args.mode, tokenizer_conf=dict(token_list=token_list(cfg.vocab_size)), **cfg.reference_kwargs())
    am.model.load_state_dict(sd)
    B, T = int(feats.shape[0]), int(feats.shape[1])
    kw = dict(input=feats, input_len=lens, data_type="fbank", batch_size=B)
    for _ in range(2):
        res = am.generate(**kw)
    torch.cuda.synchronize()
    steps = max(1, args.steps)
    t0 = time.perf_counter()
    for _ in range(steps):
        res = am.generate(**kw)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return {"workload": f"AutoModel.generate(fbank [{B},{T},560], data_type='fbank', batch_size={B}) with a "
                        f"{cfg.vocab_size}-token CharTokenizer: decode + readback + detokenise + sentence_postprocess "
                        "+ result dicts (reference auto_model.py:343-348)",
            "value": round(B * T * FRAME_SEC / dt, 1), "unit": "audio-sec/sec", "ms_per_step": round(dt * 1e3, 3),
            "results": len(res), "chars_mean": round(float(np.mean([len(r["text"]) for r in res])), 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--mode", default="fast", choices=["fast", "exact"])
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--frames", type=int, default=500)
    ap.add_argument("--cpu-utts", type=int, default=64, help="cpu_baseline sample size (0 = skip; default the whole B=64)")
    ap.add_argument("--strong", type=int, default=0, metavar="GLOBAL_B",
                    help="strong scaling: GLOBAL_B utterances in total (BASELINE C3: 512), split over the ranks")
    ap.add_argument("--exact-steps", type=int, default=2, help="timed exact-mode steps (0 = skip)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--sv-steps", type=int, default=3, help="timed SenseVoiceSmall (config C4) steps (0 = skip)")
    ap.add_argument("--stream-chunks", type=int, default=50,
                    help="600 ms chunks per stream in the streaming (config C5) leg (0 = skip)")
    ap.add_argument("--stream-batch", type=int, default=64, help="concurrent streams of the C5 serving line")
    ap.add_argument("--punc-steps", type=int, default=5, help="timed CT-Transformer punctuation calls (0 = skip)")
    ap.add_argument("--beam-steps", type=int, default=2,
                    help="timed joint decoder + CTC prefix beam search steps (Paraformer-large + CTC head; 0 = skip)")
    ap.add_argument("--beam", type=int, default=10, help="beam size of the beam-search leg")
    ap.add_argument("--generate", type=int, default=1, help="time AutoModel.generate on the headline batch (0 = skip)")
    ap.add_argument("--long-audio-s", type=int, default=300,
                    help="seconds of synthetic audio for the VAD + ASR + punctuation leg (0 = skip)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from funasr_amd.config import paraformer_large
    from funasr_amd.distributed import broadcast_state_dict
    from funasr_amd.runtime import PfmEngine
    from funasr_amd.weights import make_weights, param_layout

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        # one process per GPU: N GPUs means N ranks launched by torch.distributed.run, never a silent 1-GPU run
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch N>1 as "
                 f"python -m torch.distributed.run --nproc-per-node {args.gpus} --master-addr 127.0.0.1 "
                 f"bench.py --gpus {args.gpus}")
    # one rank per GPU over RCCL ("nccl"). PFM_DIST_BACKEND=gloo with more ranks than GPUs (ranks share a device:
    # local rank mod device count) rehearses the N > 1 code path on a one-GPU box; it is never a measurement.
    backend = os.environ.get("PFM_DIST_BACKEND", "nccl")
    gpu = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    if world > 1:
        torch.cuda.set_device(gpu)
        dist.init_process_group(backend)
    dev = torch.device("cuda", gpu)
    cfg = paraformer_large()
    B, T = args.batch, args.frames
    if args.strong > 0:   # fixed total work: this rank's share of GLOBAL_B (all T=500, so contiguous shares balance)
        from funasr_amd.distributed import shard_range
        lo, hi = shard_range(args.strong, world, rank)
        B = hi - lo
    # ranks that share a GPU (the gloo rehearsal on a one-GPU box) are a code-path check, never an N-GPU number
    n_dev = min(world, max(1, torch.cuda.device_count())) if backend == "gloo" else world
    shared = n_dev < world

    # ---- weights: generated on rank 0, one RCCL broadcast (outside the timed region)
    t0 = time.time()
    eng = PfmEngine(cfg, gpu)
    if world > 1:   # one flat RCCL broadcast, set straight from device memory (pfm_set_weight_device)
        bdev = dev if backend != "gloo" else torch.device("cpu")
        # fast mode reads every matrix as bf16: send those as bf16 (520 instead of 880 MB over xGMI)
        wire = "bf16" if args.mode == "fast" else "f32"
        flat, wire_xw = broadcast_state_dict(param_layout(cfg), make_weights(cfg, args.seed) if rank == 0 else None,
                                             device=bdev, keep_on_device=True, wire=wire, with_xw=True)
        eng.load_flat_device(flat.to(dev), param_layout(cfg), fast_only=wire == "bf16", wire_xw=wire_xw)
        sd = None   # the host-side legs (long audio, CPU baseline) run at N=1 only
        del flat
    else:
        sd = make_weights(cfg, args.seed)
        eng.load_state_dict(sd)
    eng.reserve(B, T)
    t_setup = time.time() - t0

    # ---- synthetic fbank batch resident in HBM (distinct per rank)
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    feats = torch.randn((B, T, cfg.input_size), generator=g, device=dev, dtype=torch.float32)
    lens = torch.full((B,), T, dtype=torch.int32, device=dev)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        eng.run(feats, lens, mode=args.mode)
    torch.cuda.synchronize()

    # pass 1 (headline): K uninstrumented steps -> value / ms_per_step
    barrier()
    torch.cuda.synchronize()
    ts = time.perf_counter()
    last = None
    for _ in range(args.steps):
        last = eng.run(feats, lens, mode=args.mode)
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - ts
    # pass 2 (roofline): the same K steps with live HIP events around every GEMM / attention launch on
    # the launch stream. The events add ~2 ms of queue gaps per step, so they stay out of pass 1.
    eng.profile(True)
    torch.cuda.synchronize()
    ti = time.perf_counter()
    for _ in range(args.steps):
        eng.run(feats, lens, mode=args.mode)
    torch.cuda.synchronize()
    dt_instr = time.perf_counter() - ti
    gemm = eng.profile_read(0)
    attn = eng.profile_read(1)
    dom = eng.profile_read(3)   # the dominant kernel alone (ffn2_kernel<4>, also inside class 0)
    eng.profile(False)
    # event-pair overhead on the launch stream (record -> record with nothing between), averaged over
    # 256 pairs queued behind real work; subtracted from each bracketed launch (reported raw as well)
    pairs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(256)]
    eng.run(feats, lens, mode=args.mode)
    for a, b in pairs:
        a.record()
        b.record()
    torch.cuda.synchronize()
    ev_over_ms = float(np.median([a.elapsed_time(b) for a, b in pairs]))
    B_all = B
    if world > 1:
        cdev = "cpu" if backend == "gloo" else dev
        t = torch.tensor([dt], dtype=torch.float64, device=cdev)
        nb = torch.tensor([B], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(nb, op=dist.ReduceOp.SUM)
        dt, B_all = float(t.item()), int(nb.item())

    ntok = last["ntok"].cpu().numpy()
    audio_s = B_all * T * FRAME_SEC * args.steps
    value = audio_s / dt
    step_ms = dt / args.steps * 1000.0
    fl_step = path_flops(T, ntok)
    peak = PEAK_TFLOPS[args.mode]
    g_raw_ms = gemm["ms"]
    gemm["ms"] = max(1e-9, gemm["ms"] - ev_over_ms * gemm["launches"])
    attn["ms"] = max(1e-9, attn["ms"] - ev_over_ms * attn["launches"])
    d_raw_ms = dom["ms"]
    dom["ms"] = max(1e-9, dom["ms"] - ev_over_ms * dom["launches"])
    g_ach = gemm["flops"] / (gemm["ms"] / 1e3) / 1e12 if gemm["ms"] > 0 else 0.0
    # HBM bytes per launch of the same kernel set from the committed PMC passes (rocprofv3 --pmc FETCH_SIZE /
    # WRITE_SIZE, separate runs of this bench, gfx950-corrected by tools/pmc_traffic.py); null when absent
    # and the class's MFMA-busy fraction from a third pass (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE)
    traffic, traffic_src, busy, busy_src = None, None, None, None
    tname = next((n for n in ("r06_pmc_bench.json", "r05_pmc_bench.json", "r04_pmc_bench.json", "r03_gemm_traffic.json", "r02b_gemm_traffic.json")
                  if os.path.exists(os.path.join(ROOT, "profiles", n))), None)
    if args.mode == "fast" and tname:
        with open(os.path.join(ROOT, "profiles", tname)) as f:
            pmc = json.load(f)
        traffic = round(pmc["hbm_bytes_per_launch"])
        traffic_src = (f"profiles/{tname} (PMC FETCH_SIZE x2 + WRITE_SIZE per launch of the GEMM "
                       "class: bf16 GEMMs + fused FFN)")
        if pmc.get("mfma_busy_gemm_class") is not None:
            busy = round(pmc["mfma_busy_gemm_class"], 4)
            busy_src = f"profiles/{tname}: " + pmc.get("mfma_busy_definition", "")
    from funasr_amd.distributed import fast_xw_bits
    xw_bits = fast_xw_bits()
    # the encoder layer launch: MODE 4, or with PFM_FAST_XW bit 4 / 8 MODE 5 / 6 (the v rows' / Wo's second weight
    # plane streamed too; algorithmic FLOPs are the same)
    dom_kernel = "ffn2_kernel<%d>" % (6 if xw_bits & 8 else 5 if xw_bits & 4 else 4)
    roofline = {"bound": "mfma",
                "kernel": (f"{dom_kernel} (encoder out-proj + LN2-FFN + LN1 + next QKV) + ffn_fused_kernel (decoder "
                           "FFNs) + gemm_bf16_kernel (layer-0 QKV / decoder / vocabulary)") if args.mode == "fast" else
                          "gemm_bf16_kernel, split-bf16 x6 emulation of f32 (flops counted as f32 2MNK)",
                "achieved": round(g_ach, 2), "peak": peak, "unit": "TFLOP/s", "frac": round(g_ach / peak, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "mfma_busy": busy,
                "mfma_busy_source": busy_src,
                "algorithmic_bytes_per_launch": round(gemm["bytes"] / max(1, gemm["launches"])),
                "avg_launch_us": round(gemm["ms"] * 1e3 / max(1, gemm["launches"]), 2),
                "avg_launch_us_raw": round(g_raw_ms * 1e3 / max(1, gemm["launches"]), 2),
                "event_pair_overhead_us": round(ev_over_ms * 1e3, 2),
                "launches": int(gemm["launches"]), "share_of_step": round(gemm["ms"] / args.steps / step_ms, 3),
                "instrumented_ms_per_step": round(dt_instr / args.steps * 1000.0, 3),
                # the single dominant kernel, beside the class figure above: the encoder layer launch
                # ffn2_kernel<4> (out-proj + LN2-FFN + LN1 + the next layer's QKV), 2 M 512 (512 + 2048 + 2048 + 1536)
                # FLOP per launch at M = B T rows, live HIP events on its launch stream
                "dominant": ({"kernel": dom_kernel, "launches": int(dom["launches"]),
                              "gflop_per_launch": round(dom["flops"] / dom["launches"] / 1e9, 2),
                              "avg_launch_us": round(dom["ms"] * 1e3 / dom["launches"], 2),
                              "avg_launch_us_raw": round(d_raw_ms * 1e3 / dom["launches"], 2),
                              "achieved": round(dom["flops"] / (dom["ms"] / 1e3) / 1e12, 2), "peak": peak,
                              "unit": "TFLOP/s",
                              "frac": round(dom["flops"] / (dom["ms"] / 1e3) / 1e12 / peak, 4),
                              "share_of_step": round(dom["ms"] / args.steps / step_ms, 3)}
                             if dom["launches"] else None),
                "achieved_hbm_gbs": round(gemm["bytes"] / (gemm["ms"] / 1e3) / 1e9, 1) if gemm["ms"] > 0 else None}
    a_ach = attn["flops"] / (attn["ms"] / 1e3) / 1e12 if attn["ms"] > 0 else 0.0
    path_tf = fl_step / (step_ms / 1e3) / 1e12
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "audio-sec/sec", "n_gpus": n_dev, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_ms, 3), "higher_is_better": True,
        "scaling": "strong" if args.strong > 0 else "weak",
        "vs_baseline": None, "dtype": "bf16" if args.mode == "fast" else "f32",
        "data": (f"synthetic N(0,1) fbank [{args.strong},500,560] in total, split over the ranks" if args.strong > 0 else
                 f"synthetic N(0,1) fbank [{B},500,560] per GPU") + ", seeded random-init Paraformer-large weights",
        "config": {"workload": (f"Paraformer-large offline batch, {args.strong} x 30 s (T=500 LFR frames) fbank in "
                                "total (strong scaling)") if args.strong > 0 else
                               f"Paraformer-large offline batch, B={B} x 30 s (T=500 LFR frames) fbank per GPU",
                   "global_batch": B_all, "frames": T, "parallelism": f"dp{world}", "mode": args.mode,
                   "tokens_per_utt_mean": float(ntok.mean()),
                   # fast = bf16 operands: NOT token-exact vs the f32 CPU reference (flips only where the
                   # reference top-2 margin < 0.5 nat, tests/test_gpu_parity.py); exact = token-exact
                   "token_exact": args.mode == "exact"},
        "roofline": roofline,
        "attention": {"achieved": round(a_ach, 2), "unit": "TFLOP/s",
                      "share_of_step": round(attn["ms"] / args.steps / step_ms, 3)},
        "path_roofline": {"bound": "mfma", "achieved": round(path_tf, 2), "peak": peak, "unit": "TFLOP/s",
                          "frac": round(path_tf / peak, 4), "gflop_per_audio_sec": round(fl_step / (B * T * FRAME_SEC) / 1e9, 3)},
        "setup_s": round(t_setup, 2),
    }
    if world > 1:
        out["ranks"] = world
        out["shared_device"] = shared
        if shared:   # not an N-GPU result: N ranks time-share fewer devices
            out["metric"] = METRIC + " [REHEARSAL: ranks share a device, not a multi-GPU measurement]"

    # fast-mode fidelity of the benched dispatch on the reference's own B = 64 x 500 run (tests/golden/para_large_b64:
    # per-position top-5 log-probs of the reference decoder; regret statistics of tests/fast_parity.py) beside the
    # CPU emulation of ideal bf16 operands (tests/golden/fast_emul.json)
    if rank == 0 and world == 1 and args.mode == "fast":
        gpath = os.path.join(ROOT, "tests", "golden", "para_large_b64.npz")
        if os.path.exists(gpath):
            from tests.fast_parity import paraformer_stats
            from tests.golden.inputs import fbank_input
            gg = np.load(gpath)
            gx, gl = fbank_input(int(gg["seed"]), int(gg["B"]), int(gg["T"]), gg["lens"])
            rr = eng.run(torch.from_numpy(gx).to(dev), torch.from_numpy(gl).to(dev), mode="fast")
            st = paraformer_stats(rr["tokens"].cpu().numpy(), rr["ntok"].cpu().numpy(), gg, 0.5)
            em = json.load(open(os.path.join(ROOT, "tests", "golden", "fast_emul.json")))["para_large_b64"]
            out["fast_fidelity"] = {
                "golden": "para_large_b64 (reference run, B=64 x 500, seeded weights)",
                "pfm_fast_xw": fast_xw_bits(),
                "flip_frac": round(st["flip_frac"], 4), "mean_regret_nat": round(st["mean_regret"], 5),
                "max_regret_nat": round(st["max_regret"], 4),
                "outside_top5_frac": round(st["outside_topk"] / max(1, st["positions"]), 5),
                "equal_token_counts": round(st["equal_counts"], 4),
                "ideal_bf16_emulation": {"flip_frac": round(em["G"]["flip_frac"], 4),
                                         "mean_regret_nat": round(em["G"]["mean_regret"], 5)}}
    if rank == 0:
        progress("headline leg done")
    # ---- exact (f32 MFMA) mode on the same batch: token-parity mode throughput + agreement
    if rank == 0 and world == 1 and args.mode == "fast" and args.exact_steps > 0:
        eng.run(feats, lens, mode="exact")
        torch.cuda.synchronize()
        te = time.perf_counter()
        for _ in range(args.exact_steps):
            ex = eng.run(feats, lens, mode="exact")
        torch.cuda.synchronize()
        dte = (time.perf_counter() - te) / args.exact_steps
        a, b = last["tokens"].cpu().numpy(), ex["tokens"].cpu().numpy()
        na, nb = last["ntok"].cpu().numpy(), ex["ntok"].cpu().numpy()
        agree = [np.mean(a[i, :min(na[i], nb[i])] == b[i, :min(na[i], nb[i])]) for i in range(B)
                 if min(na[i], nb[i]) > 0]
        fl_ex = path_flops(T, nb)
        x6 = os.environ.get("PFM_EXACT_X6", "1") != "0"
        terms = 6
        tf_ex = fl_ex / dte / 1e12
        out["exact_mode"] = {
            "value": round(B * T * FRAME_SEC / dte, 1), "ms_per_step": round(dte * 1e3, 2), "dtype": "f32",
            "token_exact": True,   # token ids identical to the reference on every golden (tests/test_gpu_parity.py)
            "arithmetic": ("split-bf16 x6 MFMA (x = x0+x1+x2 bf16, six products, f32 accumulate) for every GEMM "
                           "and the attention" if x6 else "v_mfma_f32_32x32x2_f32"),
            "path_tflops_f32_equiv": round(tf_ex, 2),
            "path_roofline": ({"bound": "mfma", "achieved": round(terms * tf_ex, 2), "peak": PEAK_TFLOPS["fast"],
                               "unit": f"TFLOP/s (bf16 MFMA issued: about {terms} x f32-equivalent)",
                               "frac": round(terms * tf_ex / PEAK_TFLOPS["fast"], 4)} if x6 else
                              {"bound": "mfma", "achieved": round(tf_ex, 2), "peak": PEAK_TFLOPS["exact"],
                               "unit": "TFLOP/s", "frac": round(tf_ex / PEAK_TFLOPS["exact"], 4)}),
            "fast_vs_exact_token_agreement": round(float(np.mean(agree)), 4),
            "fast_vs_exact_ntok_equal": round(float(np.mean(na == nb)), 4)}

    # ---- AutoModel.generate() on the same batch: the metric as SURVEY §8(d) defines it (decode + host result dicts)
    if rank == 0 and world == 1 and args.generate:
        g = generate_leg(args, sd, cfg, feats, lens)
        out["generate"] = g
        out["generate_value"] = g["value"]
    if rank == 0:
        progress("exact leg done")
    # ---- SenseVoiceSmall (BASELINE config C4): B x 30 s on the same fbank batch, rank 0
    if rank == 0 and args.sv_steps > 0:
        from funasr_amd.config import sense_voice_small
        scfg = sense_voice_small()
        seng = PfmEngine(scfg, gpu)
        seng.load_state_dict(make_weights(scfg, args.seed))
        seng.reserve(B, T + 4)
        q = [0, 1, 2, 15]   # language auto, event, emotion, woitn
        for _ in range(2):
            seng.run_ctc(feats, lens, q, mode=args.mode)
        torch.cuda.synchronize()
        tsv = time.perf_counter()
        for _ in range(args.sv_steps):
            sv_last = seng.run_ctc(feats, lens, q, mode=args.mode)
        torch.cuda.synchronize()
        dsv = (time.perf_counter() - tsv) / args.sv_steps
        sv_tf = B * sensevoice_flops(T + 4) / dsv / 1e12
        out["sensevoice"] = {"workload": f"SenseVoiceSmall B={B} x 30 s (T={T}+4 query rows), CTC greedy",
                             "value": round(B * T * FRAME_SEC / dsv, 1), "unit": "audio-sec/sec",
                             "ms_per_step": round(dsv * 1e3, 3), "dtype": out["dtype"],
                             "path_tflops": round(sv_tf, 2), "path_frac": round(sv_tf / peak, 4),
                             "tokens_per_utt_mean": float(sv_last["ntok"].float().mean().item())}
        del seng

    if rank == 0:
        progress("SenseVoice leg done")
    # ---- joint decoder + CTC prefix beam search (BASELINE config C5's CTC prefix-beam; Paraformer.inference with
    # decoding_ctc_weight): Paraformer-large with a CTC head (ctc_weight 0.3), the same batch, rank 0
    if rank == 0 and args.beam_steps > 0:
        import dataclasses
        bcfg = dataclasses.replace(cfg, ctc_weight=0.3)
        beng = PfmEngine(bcfg, gpu)
        beng.load_state_dict(make_weights(bcfg, args.seed))
        beng.reserve(B, T)
        bkw = dict(mode=args.mode, beam=args.beam, ctc_weight=0.3, penalty=0.0, nbest=1)
        beng.run_beam(feats, lens, **bkw)
        torch.cuda.synchronize()
        tb = time.perf_counter()
        for _ in range(args.beam_steps):
            bl = beng.run_beam(feats, lens, **bkw)
        torch.cuda.synchronize()
        dtb = (time.perf_counter() - tb) / args.beam_steps
        nb = bl["ntok"][:, 0].float()
        out["beam_search"] = {"workload": (f"Paraformer-large + CTC head, B={B} x 30 s, joint decoder + CTC prefix beam "
                                           f"search (beam {args.beam}, decoding_ctc_weight 0.3, pre-beam "
                                           f"{int(1.5 * args.beam)}, end detection), co-resident workgroups per utterance "
                                           f"(r^n / r^b / log-psi chains on separate SIMDs)"),
                              "value": round(B * T * FRAME_SEC / dtb, 1), "unit": "audio-sec/sec",
                              "ms_per_step": round(dtb * 1e3, 2), "dtype": out["dtype"],
                              "tokens_per_utt_mean": round(float(nb[nb >= 0].mean().item()), 2)}
        del beng

    if rank == 0:
        progress("beam-search leg done")
    # ---- streaming Paraformer (BASELINE config C5): 600 ms chunks ([0, 10, 5], look-back 4 / 1) of
    # 30 s streams through pfm_stream_step, synthetic LFR+CMVN chunk rows resident in HBM; one stream
    # (the reference's batch 1: per-chunk latency) and S concurrent streams (serving throughput), rank 0
    if rank == 0 and world == 1 and args.stream_chunks > 0:
        out["streaming"] = stream_leg(args, dev, torch, make_weights)

    if rank == 0:
        progress("streaming leg done")
    # ---- CT-Transformer punctuation: 64 word sequences x 200 words per pfm_run_punc
    if rank == 0 and world == 1 and args.punc_steps > 0:
        out["punctuation"] = punc_leg(args, dev, torch, make_weights)

    if rank == 0:
        progress("punctuation leg done")
    # ---- VAD-segmented long-audio transcription: FSMN-VAD -> ASR -> punctuation
    if rank == 0 and world == 1 and args.long_audio_s > 0:
        out["long_audio"] = long_audio_leg(args, sd, cfg)

    if rank == 0:
        progress("long-audio leg done")
    # ---- CPU baseline: the oracle torch-CPU restatement on a bounded sample (rank 0, N=1 only)
    if rank == 0 and world == 1 and args.cpu_utts > 0:
        from oracle.paraformer_ref import paraformer_infer
        torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
        x = feats[: args.cpu_utts].cpu()
        ln = lens[: args.cpu_utts].cpu()
        tc = time.perf_counter()
        paraformer_infer(x, ln, sd, cfg)
        dtc = time.perf_counter() - tc
        ncpu = os.cpu_count() or 1
        try:
            aff = len(os.sched_getaffinity(0))
        except AttributeError:
            aff = ncpu
        out["cpu_baseline"] = {"value": round(args.cpu_utts * T * FRAME_SEC / dtc, 2), "unit": "audio-sec/sec",
                               "cores": torch.get_num_threads(), "kind": "port",
                               "cores_note": (f"{torch.get_num_threads()} threads = this job's CPU share on the GPU box "
                                              f"(OMP_NUM_THREADS, the pool's per-GPU allotment); os.cpu_count() = "
                                              f"{ncpu} and sched_getaffinity = {aff} report the whole host"),
                               "sample": f"{args.cpu_utts} utts x 30 s (T=500) of the same batch, one call of "
                                         f"oracle/paraformer_ref.py (torch-CPU fp32, op-for-op restatement), "
                                         f"{dtc:.1f} s on {cpu_model()}"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
