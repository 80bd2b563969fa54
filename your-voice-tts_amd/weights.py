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
                   location_attn: bool = False, trans_agent: bool = False):
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
    add("decoder.prenet.layers.0.linear_layer.weight", (PRENET, nm), _lin(nm, PRENET))
    add("decoder.prenet.layers.1.linear_layer.weight", (PRENET, PRENET), _lin(PRENET, PRENET))
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
