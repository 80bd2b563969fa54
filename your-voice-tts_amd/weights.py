"""Parameter table of the Tacotron2 synthesis path and a deterministic weight generator.

The table lists every ``state_dict`` entry the reference ``Tacotron2`` module holds
(``models/tacotron2.py:11-45``, ``layers/tacotron2.py:9-150``,
``layers/common_layers.py:8-131``), with the initialisation bound the reference's
constructors use, so that generated weights have the same magnitudes as the reference's
random init:

* ``Linear`` (``common_layers.py:8-25``): xavier-uniform, bound = gain*sqrt(6/(fan_in+fan_out)),
  gain 1 ('linear', 'sigmoid') or 5/3 ('tanh'); bias follows ``nn.Linear``: U(+-1/sqrt(fan_in)).
* ``nn.LSTMCell`` / ``nn.LSTM``: U(+-1/sqrt(hidden)).
* ``nn.Conv1d``: U(+-1/sqrt(in_channels*kernel)) for weight and bias.
* ``nn.Embedding`` init rows (go frame, RNN inits): N(0,1) in the reference; here U(+-sqrt(3)),
  same variance.  Character embedding: U(+-sqrt(3)*sqrt(2/(num_chars+512)))
  (``models/tacotron2.py:28-31``).
* BatchNorm buffers: the reference starts at gamma=1, beta=0, mean=0, var=1; a trained
  checkpoint does not, so the generator draws gamma~U(0.8,1.2), beta,mean~U(-0.1,0.1),
  var~U(0.5,1.5) to exercise the BN arithmetic.

Every tensor is drawn from its own PCG64 stream seeded with ``seed ^ crc32(key)``, so the
values depend only on (seed, key, shape): the GPU box regenerates the exact weights the golden
fixtures were produced with, without any reference code.
"""
from __future__ import annotations

import math
import zlib
from collections import OrderedDict

import numpy as np

TANH_GAIN = 5.0 / 3.0

# Decoder geometry fixed by the reference (layers/tacotron2.py:102-110, common_layers.py:121-131).
ENC_DIM = 512          # encoder embedding / memory width
ATT_RNN = 1024         # attention_rnn_dim
DEC_RNN = 1024         # decoder_rnn_dim
PRENET = 256           # prenet_dim
ATT_DIM = 128          # attention_dim
LOC_FILTERS = 32       # attention_location_n_filters
LOC_KERNEL = 31        # attention_location_kernel_size
N_MEL = 80
POSTNET_CH = 512
POSTNET_K = 5
N_POSTNET = 5


def _lin(fan_in, fan_out, gain=1.0):
    return ("uniform", gain * math.sqrt(6.0 / (fan_in + fan_out)))


def tacotron2_spec(num_chars: int = 130, num_speakers: int = 0, r: int = 1,
                   location_attn: bool = False, trans_agent: bool = False, prenet_bn: bool = False):
    """Ordered list of (key, shape, (kind, arg)) in the reference ``state_dict`` order."""
    s = []
    add = lambda k, shape, init: s.append((k, tuple(shape), init))
    emb_b = math.sqrt(3.0) * math.sqrt(2.0 / (num_chars + 512))
    add("embedding.weight", (num_chars, 512), ("uniform", emb_b))
    if num_speakers > 1:
        # models/tacotron2.py:32-34: normal(0, 0.3) -> same-variance uniform
        add("speaker_embedding.weight", (num_speakers, 512), ("uniform", 0.3 * math.sqrt(3.0)))

    def conv_bn(prefix, cin, cout, k):
        b = 1.0 / math.sqrt(cin * k)
        add(prefix + ".net.0.weight", (cout, cin, k), ("uniform", b))
        add(prefix + ".net.0.bias", (cout,), ("uniform", b))
        add(prefix + ".net.1.weight", (cout,), ("range", (0.8, 1.2)))
        add(prefix + ".net.1.bias", (cout,), ("uniform", 0.1))
        add(prefix + ".net.1.running_mean", (cout,), ("uniform", 0.1))
        add(prefix + ".net.1.running_var", (cout,), ("range", (0.5, 1.5)))
        add(prefix + ".net.1.num_batches_tracked", (), ("zero_i64", None))

    for i in range(3):
        conv_bn(f"encoder.convolutions.{i}", 512, 512, 5)
    hb = 1.0 / math.sqrt(256)
    for sfx in ("", "_reverse"):
        add(f"encoder.lstm.weight_ih_l0{sfx}", (1024, 512), ("uniform", hb))
        add(f"encoder.lstm.weight_hh_l0{sfx}", (1024, 256), ("uniform", hb))
        add(f"encoder.lstm.bias_ih_l0{sfx}", (1024,), ("uniform", hb))
        add(f"encoder.lstm.bias_hh_l0{sfx}", (1024,), ("uniform", hb))

    nm = N_MEL * r
    for i, nin in enumerate((nm, PRENET)):
        add(f"decoder.prenet.layers.{i}.linear_layer.weight", (PRENET, nin), _lin(nin, PRENET))
        if prenet_bn:  # LinearBN (common_layers.py:27-52): BatchNorm1d over the layer's outputs
            pb = f"decoder.prenet.layers.{i}.bn."
            add(pb + "weight", (PRENET,), ("range", (0.8, 1.2)))
            add(pb + "bias", (PRENET,), ("uniform", 0.1))
            add(pb + "running_mean", (PRENET,), ("uniform", 0.1))
            add(pb + "running_var", (PRENET,), ("range", (0.5, 1.5)))
            add(pb + "num_batches_tracked", (), ("zero_i64", None))
    ab = 1.0 / math.sqrt(ATT_RNN)
    add("decoder.attention_rnn.weight_ih", (4 * ATT_RNN, PRENET + ENC_DIM), ("uniform", ab))
    add("decoder.attention_rnn.weight_hh", (4 * ATT_RNN, ATT_RNN), ("uniform", ab))
    add("decoder.attention_rnn.bias_ih", (4 * ATT_RNN,), ("uniform", ab))
    add("decoder.attention_rnn.bias_hh", (4 * ATT_RNN,), ("uniform", ab))
    add("decoder.attention_layer.query_layer.linear_layer.weight", (ATT_DIM, ATT_RNN),
        _lin(ATT_RNN, ATT_DIM, TANH_GAIN))
    add("decoder.attention_layer.inputs_layer.linear_layer.weight", (ATT_DIM, ENC_DIM),
        _lin(ENC_DIM, ATT_DIM, TANH_GAIN))
    add("decoder.attention_layer.v.linear_layer.weight", (1, ATT_DIM), _lin(ATT_DIM, 1))
    add("decoder.attention_layer.v.linear_layer.bias", (1,), ("uniform", 1.0 / math.sqrt(ATT_DIM)))
    if trans_agent:
        tb = 1.0 / math.sqrt(ATT_RNN + ENC_DIM)
        add("decoder.attention_layer.ta.weight", (1, ATT_RNN + ENC_DIM), ("uniform", tb))
        add("decoder.attention_layer.ta.bias", (1,), ("uniform", tb))
    if location_attn:
        add("decoder.attention_layer.location_layer.location_conv.weight",
            (LOC_FILTERS, 2, LOC_KERNEL), ("uniform", 1.0 / math.sqrt(2 * LOC_KERNEL)))
        add("decoder.attention_layer.location_layer.location_dense.linear_layer.weight",
            (ATT_DIM, LOC_FILTERS), _lin(LOC_FILTERS, ATT_DIM, TANH_GAIN))
    db = 1.0 / math.sqrt(DEC_RNN)
    add("decoder.decoder_rnn.weight_ih", (4 * DEC_RNN, ATT_RNN + ENC_DIM), ("uniform", db))
    add("decoder.decoder_rnn.weight_hh", (4 * DEC_RNN, DEC_RNN), ("uniform", db))
    add("decoder.decoder_rnn.bias_ih", (4 * DEC_RNN,), ("uniform", db))
    add("decoder.decoder_rnn.bias_hh", (4 * DEC_RNN,), ("uniform", db))
    add("decoder.linear_projection.linear_layer.weight", (nm, DEC_RNN + ENC_DIM),
        _lin(DEC_RNN + ENC_DIM, nm))
    add("decoder.linear_projection.linear_layer.bias", (nm,),
        ("uniform", 1.0 / math.sqrt(DEC_RNN + ENC_DIM)))
    add("decoder.stopnet.1.linear_layer.weight", (1, DEC_RNN + nm), _lin(DEC_RNN + nm, 1))
    add("decoder.stopnet.1.linear_layer.bias", (1,), ("uniform", 1.0 / math.sqrt(DEC_RNN + nm)))
    add("decoder.attention_rnn_init.weight", (1, ATT_RNN), ("uniform", math.sqrt(3.0)))
    add("decoder.go_frame_init.weight", (1, nm), ("uniform", math.sqrt(3.0)))
    add("decoder.decoder_rnn_inits.weight", (1, DEC_RNN), ("uniform", math.sqrt(3.0)))

    chans = [N_MEL] + [POSTNET_CH] * (N_POSTNET - 1) + [N_MEL]
    for i in range(N_POSTNET):
        conv_bn(f"postnet.convolutions.{i}", chans[i], chans[i + 1], POSTNET_K)
    return s


def _default_linear(fan_in):
    """nn.Linear / nn.Conv default init (kaiming_uniform a=sqrt(5)): U(+-1/sqrt(fan_in))."""
    return ("uniform", 1.0 / math.sqrt(fan_in))


def tacotron_gst_spec(num_chars: int = 130, num_speakers: int = 0, r: int = 5, memory_size: int = 5,
                      location_attn: bool = False, trans_agent: bool = False, gst: bool = True,
                      prenet_bn: bool = False):
    """Ordered (key, shape, init) table of the reference ``TacotronGST`` (models/tacotrongst.py:10-45;
    ``gst=False`` gives the plain ``Tacotron`` of models/tacotron.py:9-43): Tacotron ``Encoder`` /
    ``CBHG`` / ``Decoder`` / ``PostCBHG`` (layers/tacotron.py:7-489) and ``GST``
    (layers/gst_layers.py:6-168).  BatchNormConv1d convs have no bias (layers/tacotron.py:36-42)."""
    s = []
    add = lambda k, shape, init: s.append((k, tuple(shape), init))
    add("embedding.weight", (num_chars, 256), ("uniform", 0.3 * math.sqrt(3.0)))  # normal(0, 0.3)
    if num_speakers > 1:
        add("speaker_embedding.weight", (num_speakers, 256), ("uniform", 0.3 * math.sqrt(3.0)))

    def bn(prefix, c):
        add(prefix + ".weight", (c,), ("range", (0.8, 1.2)))
        add(prefix + ".bias", (c,), ("uniform", 0.1))
        add(prefix + ".running_mean", (c,), ("uniform", 0.1))
        add(prefix + ".running_var", (c,), ("range", (0.5, 1.5)))
        add(prefix + ".num_batches_tracked", (), ("zero_i64", None))

    def bn_conv(prefix, cin, cout, k):
        add(prefix + ".conv1d.weight", (cout, cin, k), _default_linear(cin * k))
        bn(prefix + ".bn", cout)

    def gru(prefix, nin, h, bidir):
        b = 1.0 / math.sqrt(h)
        for sfx in ("", "_reverse") if bidir else ("",):
            add(f"{prefix}.weight_ih_l0{sfx}", (3 * h, nin), ("uniform", b))
            add(f"{prefix}.weight_hh_l0{sfx}", (3 * h, h), ("uniform", b))
            add(f"{prefix}.bias_ih_l0{sfx}", (3 * h,), ("uniform", b))
            add(f"{prefix}.bias_hh_l0{sfx}", (3 * h,), ("uniform", b))

    def cbhg(prefix, cin, K, projections):
        for k in range(1, K + 1):
            bn_conv(f"{prefix}.conv1d_banks.{k - 1}", cin, 128, k)
        ins = [K * 128] + projections[:-1]
        for i, (a, b) in enumerate(zip(ins, projections)):
            bn_conv(f"{prefix}.conv1d_projections.{i}", a, b, 3)
        if projections[-1] != 128:
            add(f"{prefix}.pre_highway.weight", (128, projections[-1]), _default_linear(projections[-1]))
        for i in range(4):
            for n in ("H", "T"):
                add(f"{prefix}.highways.{i}.{n}.weight", (128, 128), _default_linear(128))
                add(f"{prefix}.highways.{i}.{n}.bias", (128,), _default_linear(128))
        gru(f"{prefix}.gru", 128, 128, True)

    def prenet(prefix, nin, outs, with_bn=False):
        for i, (a, b) in enumerate(zip([nin] + outs[:-1], outs)):
            add(f"{prefix}.layers.{i}.linear_layer.weight", (b, a), _lin(a, b))
            add(f"{prefix}.layers.{i}.linear_layer.bias", (b,), _default_linear(a))
            if with_bn:  # LinearBN (common_layers.py:28-52)
                bn(f"{prefix}.layers.{i}.bn", b)

    prenet("encoder.prenet", 256, [256, 128])
    cbhg("encoder.cbhg.cbhg", 128, 16, [128, 128])
    if gst:
        filters = [1, 32, 32, 64, 64, 128, 128]
        for i in range(6):
            add(f"gst.encoder.convs.{i}.weight", (filters[i + 1], filters[i], 3, 3), _default_linear(filters[i] * 9))
            add(f"gst.encoder.convs.{i}.bias", (filters[i + 1],), _default_linear(filters[i] * 9))
        for i in range(6):
            bn(f"gst.encoder.bns.{i}", filters[i + 1])
        gru("gst.encoder.recurrence", 256, 128, False)
        add("gst.style_token_layer.style_tokens", (10, 64), ("uniform", math.sqrt(3.0) / 8.0))  # orthogonal rows
        add("gst.style_token_layer.attention.W_query.weight", (256, 128), _default_linear(128))
        add("gst.style_token_layer.attention.W_key.weight", (256, 64), _default_linear(64))
        add("gst.style_token_layer.attention.W_value.weight", (256, 64), _default_linear(64))
    mem = 80 * memory_size
    prenet("decoder.prenet", mem, [256, 128], prenet_bn)  # prenet_type (layers/tacotron.py:283-287)
    hb = 1.0 / math.sqrt(256)
    add("decoder.attention_rnn.weight_ih", (768, 384), ("uniform", hb))
    add("decoder.attention_rnn.weight_hh", (768, 256), ("uniform", hb))
    add("decoder.attention_rnn.bias_ih", (768,), ("uniform", hb))
    add("decoder.attention_rnn.bias_hh", (768,), ("uniform", hb))
    add("decoder.attention_layer.query_layer.linear_layer.weight", (ATT_DIM, 256), _lin(256, ATT_DIM, TANH_GAIN))
    add("decoder.attention_layer.inputs_layer.linear_layer.weight", (ATT_DIM, 256), _lin(256, ATT_DIM, TANH_GAIN))
    add("decoder.attention_layer.v.linear_layer.weight", (1, ATT_DIM), _lin(ATT_DIM, 1))
    add("decoder.attention_layer.v.linear_layer.bias", (1,), ("uniform", 1.0 / math.sqrt(ATT_DIM)))
    if trans_agent:
        tb = 1.0 / math.sqrt(512)
        add("decoder.attention_layer.ta.weight", (1, 512), ("uniform", tb))
        add("decoder.attention_layer.ta.bias", (1,), ("uniform", tb))
    if location_attn:
        add("decoder.attention_layer.location_layer.location_conv.weight",
            (LOC_FILTERS, 2, LOC_KERNEL), ("uniform", 1.0 / math.sqrt(2 * LOC_KERNEL)))
        add("decoder.attention_layer.location_layer.location_dense.linear_layer.weight",
            (ATT_DIM, LOC_FILTERS), _lin(LOC_FILTERS, ATT_DIM, TANH_GAIN))
    add("decoder.project_to_decoder_in.weight", (256, 512), _default_linear(512))
    add("decoder.project_to_decoder_in.bias", (256,), _default_linear(512))
    for i in range(2):
        add(f"decoder.decoder_rnns.{i}.weight_ih", (768, 256), ("uniform", hb))
        add(f"decoder.decoder_rnns.{i}.weight_hh", (768, 256), ("uniform", hb))
        add(f"decoder.decoder_rnns.{i}.bias_ih", (768,), ("uniform", hb))
        add(f"decoder.decoder_rnns.{i}.bias_hh", (768,), ("uniform", hb))
    add("decoder.proj_to_mel.weight", (80 * r, 256), _default_linear(256))
    add("decoder.proj_to_mel.bias", (80 * r,), _default_linear(256))
    add("decoder.attention_rnn_init.weight", (1, 256), ("uniform", math.sqrt(3.0)))
    add("decoder.memory_init.weight", (1, mem), ("uniform", math.sqrt(3.0)))
    add("decoder.decoder_rnn_inits.weight", (2, 256), ("uniform", math.sqrt(3.0)))
    add("decoder.stopnet.linear.weight", (1, 256 + 80 * r), _lin(256 + 80 * r, 1))
    add("decoder.stopnet.linear.bias", (1,), _default_linear(256 + 80 * r))
    cbhg("postnet.cbhg", 80, 8, [256, 80])
    add("last_linear.0.weight", (1025, 256), _default_linear(256))
    add("last_linear.0.bias", (1025,), _default_linear(256))
    return s


def tacotron_gst_weights(seed: int = 0, **spec_kw):
    return generate(tacotron_gst_spec(**spec_kw), seed)


def synthetic_style_mel(frames: int, seed: int) -> np.ndarray:
    """Seeded style mel [frames, 80] ~ U[0, 1)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.uniform(0.0, 1.0, size=(frames, N_MEL)).astype(np.float32)


def generate(spec, seed: int = 0) -> "OrderedDict[str, np.ndarray]":
    """Deterministic weights for ``spec``: one PCG64 stream per key, seeded seed ^ crc32(key)."""
    out = OrderedDict()
    for key, shape, (kind, arg) in spec:
        rng = np.random.Generator(np.random.PCG64((seed ^ zlib.crc32(key.encode())) & 0xFFFFFFFF))
        if kind == "uniform":
            v = rng.uniform(-arg, arg, size=shape)
        elif kind == "range":
            v = rng.uniform(arg[0], arg[1], size=shape)
        elif kind == "zero_i64":
            out[key] = np.zeros(shape, dtype=np.int64)
            continue
        else:
            raise ValueError(kind)
        out[key] = np.asarray(v, dtype=np.float32)
    return out


def tacotron2_weights(seed: int = 0, **spec_kw):
    return generate(tacotron2_spec(**spec_kw), seed)


def synthetic_ids(L: int, seed: int, num_chars: int = 130) -> np.ndarray:
    """Seeded character ids ~ U{3..num_chars-1}."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.integers(3, num_chars, size=L, dtype=np.int64)


def synthetic_lengths(B: int, seed: int, lo: int = 60, hi: int = 160) -> np.ndarray:
    """Per-sentence encoder lengths L_b ~ U{lo..hi}."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.integers(lo, hi + 1, size=B, dtype=np.int64)
