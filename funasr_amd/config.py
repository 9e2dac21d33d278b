"""Paraformer model configuration (the shapes the HIP path is built for).

Mirrors the reference template `funasr/models/paraformer/template.yaml:8-66`
(encoder_conf / decoder_conf / predictor_conf / frontend_conf) and the kwarg
names AutoModel passes to the model constructor
(`funasr/auto/auto_model.py:262-265`).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Any, Dict, List


@dataclass
class FrontendConf:
    """`frontend_conf` of `funasr/frontends/wav_frontend.py:80-97` (offline WavFrontend)."""
    fs: int = 16000
    window: str = "hamming"
    n_mels: int = 80
    frame_length: int = 25          # ms
    frame_shift: int = 10           # ms
    lfr_m: int = 7
    lfr_n: int = 6
    dither: float = 0.0             # reference default 1.0; parity/golden runs force 0 (C++ runtime does too)
    cmvn_file: str | None = None
    upsacle_samples: bool = True    # (sic) reference spelling, wav_frontend.py:96


@dataclass
class ParaformerConfig:
    """Dimensions of a Paraformer (SAN-M encoder + CIF + SAN-M NAR decoder).

    Defaults are Paraformer-large (220.08M params).
    """
    input_size: int = 560           # 80 mel x lfr_m 7
    d_model: int = 512              # encoder_conf.output_size
    heads: int = 4
    ffn: int = 2048                 # linear_units
    enc_blocks: int = 50            # 1 (encoders0) + 49 (encoders)
    dec_blocks: int = 16            # att_layer_num == num_blocks -> decoders2 is None
    kernel_size: int = 11           # FSMN depthwise kernel (encoder and decoder)
    enc_sanm_shift: int = 0
    dec_sanm_shift: int = 0
    vocab_size: int = 8404
    cif_l_order: int = 1
    cif_r_order: int = 1
    cif_threshold: float = 1.0
    tail_threshold: float = 0.45
    smooth_factor: float = 1.0
    noise_threshold: float = 0.0
    ln_eps: float = 1e-12           # funasr/models/transformer/layer_norm.py:24
    blank_id: int = 0
    sos: int = 1
    eos: int = 2
    # model_conf.ctc_weight: > 0 means the model carries the CTC head ctc.ctc_lo (paraformer/model.py:95-100,
    # 147-150), which the joint CTC prefix beam search needs. The released Paraformer-large configs set 0.0;
    # the reference constructor's own default is 0.5, so pass it explicitly when a checkpoint has the head.
    ctc_weight: float = 0.0

    @property
    def d_k(self) -> int:
        return self.d_model // self.heads

    input_layer = "pe"              # class constant (SinusoidalPositionEncoder), not a field

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    @classmethod
    def from_kwargs(cls, **kw) -> "ParaformerConfig":
        """Build from AutoModel-style kwargs (encoder_conf/decoder_conf/predictor_conf)."""
        c = cls()
        enc = kw.get("encoder_conf") or {}
        dec = kw.get("decoder_conf") or {}
        pred = kw.get("predictor_conf") or {}
        if "input_size" in kw and kw["input_size"]:
            c.input_size = int(kw["input_size"])
        if "vocab_size" in kw and kw["vocab_size"] and int(kw["vocab_size"]) > 0:
            c.vocab_size = int(kw["vocab_size"])
        c.d_model = int(enc.get("output_size", c.d_model))
        c.heads = int(enc.get("attention_heads", c.heads))
        c.ffn = int(enc.get("linear_units", c.ffn))
        c.enc_blocks = int(enc.get("num_blocks", c.enc_blocks))
        c.kernel_size = int(enc.get("kernel_size", c.kernel_size))
        c.enc_sanm_shift = int(enc.get("sanm_shfit", c.enc_sanm_shift))
        if enc.get("input_layer", cls.input_layer) != cls.input_layer:
            raise ValueError(f"only input_layer='{cls.input_layer}' is on the HIP path of {cls.__name__}")
        if not enc.get("normalize_before", True):
            raise ValueError("only normalize_before=True is on the HIP path")
        nb = int(dec.get("num_blocks", c.dec_blocks))
        att = int(dec.get("att_layer_num", nb))
        if nb != att:
            raise ValueError("decoders2 (num_blocks > att_layer_num) is not on the Paraformer-large path")
        c.dec_blocks = att
        if int(dec.get("linear_units", c.ffn)) != c.ffn:
            raise ValueError("decoder linear_units must equal encoder linear_units")
        if int(dec.get("kernel_size", c.kernel_size)) != c.kernel_size:
            raise ValueError("decoder kernel_size must equal encoder kernel_size")
        c.dec_sanm_shift = int(dec.get("sanm_shfit", c.dec_sanm_shift))
        c.cif_l_order = int(pred.get("l_order", c.cif_l_order))
        c.cif_r_order = int(pred.get("r_order", c.cif_r_order))
        c.cif_threshold = float(pred.get("threshold", c.cif_threshold))
        c.tail_threshold = float(pred.get("tail_threshold", c.tail_threshold))
        c.smooth_factor = float(pred.get("smooth_factor", c.smooth_factor))
        c.noise_threshold = float(pred.get("noise_threshold", c.noise_threshold))
        for k in ("blank_id", "sos", "eos"):
            if k in kw and kw[k] is not None:
                setattr(c, k, int(kw[k]))
        if kw.get("ctc_weight") is not None:
            c.ctc_weight = float(kw["ctc_weight"])
            if c.ctc_weight >= 1.0:
                raise ValueError("ctc_weight 1.0 (a CTC-only model without decoder) is not on the HIP Paraformer path")
        return c

    def reference_kwargs(self) -> Dict[str, Any]:
        """The AutoModel / Paraformer constructor kwargs that describe this config."""
        return dict(
            encoder="SANMEncoder",
            encoder_conf=dict(output_size=self.d_model, attention_heads=self.heads,
                              linear_units=self.ffn, num_blocks=self.enc_blocks,
                              dropout_rate=0.1, positional_dropout_rate=0.1,
                              attention_dropout_rate=0.1, input_layer="pe",
                              pos_enc_class="SinusoidalPositionEncoder", normalize_before=True,
                              kernel_size=self.kernel_size, sanm_shfit=self.enc_sanm_shift,
                              selfattention_layer_type="sanm"),
            decoder="ParaformerSANMDecoder",
            decoder_conf=dict(attention_heads=self.heads, linear_units=self.ffn,
                              num_blocks=self.dec_blocks, dropout_rate=0.1,
                              positional_dropout_rate=0.1, self_attention_dropout_rate=0.1,
                              src_attention_dropout_rate=0.1, att_layer_num=self.dec_blocks,
                              kernel_size=self.kernel_size, sanm_shfit=self.dec_sanm_shift),
            predictor="CifPredictorV2",
            predictor_conf=dict(idim=self.d_model, threshold=self.cif_threshold,
                                l_order=self.cif_l_order, r_order=self.cif_r_order,
                                tail_threshold=self.tail_threshold),
            input_size=self.input_size,
            vocab_size=self.vocab_size,
        )


def paraformer_large() -> ParaformerConfig:
    return ParaformerConfig()


def paraformer_tiny(enc_blocks: int = 3, dec_blocks: int = 2, vocab_size: int = 8404) -> ParaformerConfig:
    """Reduced-depth config used for full-tensor golden vectors (same widths as large)."""
    return ParaformerConfig(enc_blocks=enc_blocks, dec_blocks=dec_blocks, vocab_size=vocab_size)


@dataclass
class ParaformerStreamingConfig(ParaformerConfig):
    """Streaming Paraformer-large (paraformer_streaming/template.yaml): the Paraformer state_dict
    with SANMEncoderChunkOpt (input_layer pe_online = StreamSinusoidalPositionEncoder,
    scama/encoder.py:188) and a causal decoder FSMN (decoder sanm_shfit 5 -> left pad 10)."""
    dec_sanm_shift: int = 5
    input_layer = "pe_online"

    def reference_kwargs(self) -> Dict[str, Any]:
        kw = super().reference_kwargs()
        kw["encoder"] = "SANMEncoderChunkOpt"
        kw["encoder_conf"].update(input_layer="pe_online", chunk_size=[12, 15], stride=[8, 10], pad_left=[0, 0],
                                  encoder_att_look_back_factor=[4, 4], decoder_att_look_back_factor=[1, 1])
        return kw


def paraformer_streaming() -> ParaformerStreamingConfig:
    return ParaformerStreamingConfig()


def paraformer_streaming_tiny(enc_blocks: int = 3, dec_blocks: int = 2,
                              vocab_size: int = 8404) -> ParaformerStreamingConfig:
    return ParaformerStreamingConfig(enc_blocks=enc_blocks, dec_blocks=dec_blocks, vocab_size=vocab_size)


@dataclass
class SenseVoiceConfig:
    """Dimensions of SenseVoiceSmall (SAN-M encoder x 50 + tp encoder x 20 + CTC head).

    Mirrors `SenseVoiceEncoderSmall.__init__` (funasr/models/sense_voice/model.py:452-548) and
    `SenseVoiceSmall.__init__` (:592-663): LayerNorm is nn.LayerNorm (eps 1e-5, :275-287), the
    four query rows come from `embed` = Embedding(7 + len(lid_dict) + len(textnorm_dict), 560)
    (:646-648), the CTC head is `ctc.ctc_lo` Linear(512, vocab) (funasr/models/ctc/ctc.py:33).
    Vocabulary 25,055 (runtime/triton_gpu/model_repo_sense_voice_small/encoder/config.pbtxt:51).
    """
    input_size: int = 560
    d_model: int = 512
    heads: int = 4
    ffn: int = 2048
    enc_blocks: int = 50            # 1 (encoders0) + 49 (encoders)
    tp_blocks: int = 20
    kernel_size: int = 11
    enc_sanm_shift: int = 0
    vocab_size: int = 25055
    n_embed: int = 16               # 7 + 7 languages + 2 text-norm styles
    ln_eps: float = 1e-5
    blank_id: int = 0
    sos: int = 1
    eos: int = 2
    # SenseVoiceSmall.__init__ :638-656 (query ids and special token ids)
    lid_dict: Dict[str, int] = field(default_factory=lambda: {"auto": 0, "zh": 3, "en": 4, "yue": 7, "ja": 11,
                                                              "ko": 12, "nospeech": 13})
    textnorm_dict: Dict[str, int] = field(default_factory=lambda: {"withitn": 14, "woitn": 15})
    emo_unk: int = 25009

    @property
    def d_k(self) -> int:
        return self.d_model // self.heads

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    @classmethod
    def from_kwargs(cls, **kw) -> "SenseVoiceConfig":
        c = cls()
        enc = kw.get("encoder_conf") or {}
        if "input_size" in kw and kw["input_size"]:
            c.input_size = int(kw["input_size"])
        if "vocab_size" in kw and kw["vocab_size"] and int(kw["vocab_size"]) > 0:
            c.vocab_size = int(kw["vocab_size"])
        c.d_model = int(enc.get("output_size", c.d_model))
        c.heads = int(enc.get("attention_heads", c.heads))
        c.ffn = int(enc.get("linear_units", c.ffn))
        c.enc_blocks = int(enc.get("num_blocks", c.enc_blocks))
        c.tp_blocks = int(enc.get("tp_blocks", c.tp_blocks))
        c.kernel_size = int(enc.get("kernel_size", c.kernel_size))
        c.enc_sanm_shift = int(enc.get("sanm_shfit", c.enc_sanm_shift))
        if not enc.get("normalize_before", True):
            raise ValueError("only normalize_before=True is on the HIP path")
        for k in ("blank_id", "sos", "eos"):
            if k in kw and kw[k] is not None:
                setattr(c, k, int(kw[k]))
        return c

    def reference_kwargs(self) -> Dict[str, Any]:
        """SenseVoiceSmall constructor kwargs (the released model's config.yaml encoder_conf)."""
        return dict(
            encoder="SenseVoiceEncoderSmall",
            encoder_conf=dict(output_size=self.d_model, attention_heads=self.heads, linear_units=self.ffn,
                              num_blocks=self.enc_blocks, tp_blocks=self.tp_blocks, dropout_rate=0.1,
                              positional_dropout_rate=0.1, attention_dropout_rate=0.1, input_layer="pe",
                              pos_enc_class="SinusoidalPositionEncoder", normalize_before=True,
                              kernel_size=self.kernel_size, sanm_shfit=self.enc_sanm_shift,
                              selfattention_layer_type="sanm"),
            input_size=self.input_size,
            vocab_size=self.vocab_size,
        )


def sense_voice_small() -> SenseVoiceConfig:
    return SenseVoiceConfig()


def sense_voice_tiny(enc_blocks: int = 3, tp_blocks: int = 2, vocab_size: int = 25055) -> SenseVoiceConfig:
    """Reduced-depth SenseVoice config for full-tensor golden vectors (same widths as Small)."""
    return SenseVoiceConfig(enc_blocks=enc_blocks, tp_blocks=tp_blocks, vocab_size=vocab_size)


@dataclass
class CTTransformerConfig:
    """CT-Transformer punctuation model (funasr/models/ct_transformer/model.py:35-79, template.yaml):
    embed Embedding(vocab, embed_unit) -> SANMEncoder (input_layer "pe", d 256, 8 heads, FFN 1024,
    4 blocks, FSMN kernel 11) -> decoder Linear(att_unit, len(punc_list)). The released model
    (punc_ct-transformer_zh-cn-common-vocab272727) has a 272,727-entry vocabulary and the full-width
    punc_list below. LayerNorm is funasr's LayerNorm (eps 1e-12)."""
    input_size: int = 256           # embed_unit (the encoder's input_size)
    d_model: int = 256              # att_unit / encoder output_size
    heads: int = 8
    ffn: int = 1024
    enc_blocks: int = 4
    kernel_size: int = 11
    enc_sanm_shift: int = 0
    vocab_size: int = 272727        # embedding rows
    ln_eps: float = 1e-12
    punc_list: List[str] = field(default_factory=lambda: ["<unk>", "_", "，", "。", "？", "、"])
    sentence_end_id: int = 3

    @property
    def d_k(self) -> int:
        return self.d_model // self.heads

    @property
    def n_punc(self) -> int:
        return len(self.punc_list)

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    @classmethod
    def from_kwargs(cls, **kw) -> "CTTransformerConfig":
        c = cls()
        enc = kw.get("encoder_conf") or {}
        if kw.get("encoder", "SANMEncoder") != "SANMEncoder":
            raise ValueError("the HIP CT-Transformer path implements encoder SANMEncoder")
        if "vocab_size" in kw and kw["vocab_size"] and int(kw["vocab_size"]) > 0:
            c.vocab_size = int(kw["vocab_size"])
        c.input_size = int(kw.get("embed_unit", enc.get("input_size", c.input_size)))
        c.d_model = int(kw.get("att_unit", enc.get("output_size", c.d_model)))
        c.heads = int(enc.get("attention_heads", c.heads))
        c.ffn = int(enc.get("linear_units", c.ffn))
        c.enc_blocks = int(enc.get("num_blocks", c.enc_blocks))
        c.kernel_size = int(enc.get("kernel_size", c.kernel_size))
        c.enc_sanm_shift = int(enc.get("sanm_shfit", c.enc_sanm_shift))
        if enc.get("input_layer", "pe") != "pe" or not enc.get("normalize_before", True):
            raise ValueError("the HIP CT-Transformer path implements input_layer pe, normalize_before True")
        if kw.get("punc_list"):
            c.punc_list = list(kw["punc_list"])
        if kw.get("sentence_end_id") is not None:
            c.sentence_end_id = int(kw["sentence_end_id"])
        return c

    def reference_kwargs(self) -> Dict[str, Any]:
        """CTTransformer constructor kwargs (template.yaml model_conf + encoder_conf)."""
        return dict(
            encoder="SANMEncoder",
            encoder_conf=dict(input_size=self.input_size, output_size=self.d_model, attention_heads=self.heads,
                              linear_units=self.ffn, num_blocks=self.enc_blocks, dropout_rate=0.1,
                              positional_dropout_rate=0.1, attention_dropout_rate=0.0, input_layer="pe",
                              pos_enc_class="SinusoidalPositionEncoder", normalize_before=True,
                              kernel_size=self.kernel_size, sanm_shfit=self.enc_sanm_shift,
                              selfattention_layer_type="sanm", padding_idx=0),
            vocab_size=self.vocab_size, punc_list=list(self.punc_list), embed_unit=self.input_size,
            att_unit=self.d_model, dropout_rate=0.1, ignore_id=0, sentence_end_id=self.sentence_end_id,
        )


def ct_transformer() -> CTTransformerConfig:
    return CTTransformerConfig()


def ct_transformer_tiny(enc_blocks: int = 2, vocab_size: int = 4000) -> CTTransformerConfig:
    """Reduced CT-Transformer for full-tensor goldens (same widths as the released model)."""
    return CTTransformerConfig(enc_blocks=enc_blocks, vocab_size=vocab_size)


@dataclass
class FsmnVADConfig:
    """FSMN-VAD (funasr/models/fsmn_vad_streaming/template.yaml; encoder.py:200-279): frames of the online
    frontend with LFR (5, 1) -> in_linear1 (400 -> 140) -> in_linear2 (-> 250) -> ReLU -> 4 x [linear (250 ->
    128, no bias) -> causal FSMN memory (lorder 20, x + sum of 20 taps) -> affine (-> 250) -> ReLU] ->
    out_linear1 (-> 140) -> out_linear2 (-> 248) -> softmax. vad_opts: VADXOptions (model.py:49-117)."""
    input_dim: int = 400
    input_affine_dim: int = 140
    fsmn_layers: int = 4
    linear_dim: int = 250
    proj_dim: int = 128
    lorder: int = 20
    rorder: int = 0
    lstride: int = 1
    output_affine_dim: int = 140
    output_dim: int = 248
    lfr_m: int = 5
    lfr_n: int = 1
    vad_opts: Dict[str, Any] = field(default_factory=lambda: dict(
        sample_rate=16000, detect_mode=1, snr_mode=0, max_end_silence_time=800, max_start_silence_time=3000,
        do_start_point_detection=True, do_end_point_detection=True, window_size_ms=200,
        sil_to_speech_time_thres=150, speech_to_sil_time_thres=150, speech_2_noise_ratio=1.0, do_extend=1,
        lookback_time_start_point=200, lookahead_time_end_point=100, max_single_segment_time=60000,
        snr_thres=-100.0, noise_frame_num_used_for_snr=100, decibel_thres=-100.0, speech_noise_thres=0.6,
        fe_prior_thres=1e-4, silence_pdf_num=1, sil_pdf_ids=[0], speech_noise_thresh_low=-0.1,
        speech_noise_thresh_high=0.3, output_frame_probs=False, frame_in_ms=10, frame_length_ms=25))

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    @classmethod
    def from_kwargs(cls, **kw) -> "FsmnVADConfig":
        c = cls()
        if kw.get("encoder", "FSMN") != "FSMN":
            raise ValueError("the HIP FSMN-VAD path implements encoder FSMN")
        enc = kw.get("encoder_conf") or {}
        for k in ("input_dim", "input_affine_dim", "fsmn_layers", "linear_dim", "proj_dim", "lorder", "rorder",
                  "lstride", "output_affine_dim", "output_dim"):
            if k in enc:
                setattr(c, k, int(enc[k]))
        if c.rorder != 0 or c.lstride != 1:
            raise ValueError("the HIP FSMN-VAD path implements rorder 0, lstride 1 (the released model)")
        fc = kw.get("frontend_conf") or {}
        c.lfr_m, c.lfr_n = int(fc.get("lfr_m", c.lfr_m)), int(fc.get("lfr_n", c.lfr_n))
        for k in list(c.vad_opts):
            if k in kw and kw[k] is not None:
                c.vad_opts[k] = kw[k]
        return c

    def reference_kwargs(self) -> Dict[str, Any]:
        return dict(encoder="FSMN", encoder_conf=dict(
            input_dim=self.input_dim, input_affine_dim=self.input_affine_dim, fsmn_layers=self.fsmn_layers,
            linear_dim=self.linear_dim, proj_dim=self.proj_dim, lorder=self.lorder, rorder=self.rorder,
            lstride=self.lstride, rstride=0, output_affine_dim=self.output_affine_dim, output_dim=self.output_dim),
            **self.vad_opts)


def fsmn_vad() -> FsmnVADConfig:
    return FsmnVADConfig()
