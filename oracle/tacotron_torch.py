"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py) — Tacotron / TacotronGST inference restated on
torch CPU, the configs[4] CPU *baseline* leg of ``bench.py`` (``cpu_baseline_gst``) and of
tools/cpu_port_vs_reference.py.

Same algorithm as ``tacotron_oracle.TacotronOracle`` (the numpy parity checker), restated as a tree of
torch ``nn`` modules named like the reference's state-dict keys (so the reference checkpoint layout
loads with ``load_state_dict``) and called in the reference's per-step order, eval-mode dropouts and
the memory-queue clone included, so that a sentence's host time matches the reference's own on the
same cores.  Nothing here is shipped: the product path never imports
``oracle/``.

Reference lines followed: ``models/tacotrongst.py:64-90`` (inference, speaker embedding),
``models/tacotron.py:59-70``; ``layers/tacotron.py:7-66`` (BatchNormConv1d), ``:69-89`` (Highway),
``:92-206`` (CBHG), ``:225-259`` (Encoder, PostCBHG), ``:262-470`` (Decoder, decode, memory queue,
inference + stop rule), ``:473-489`` (StopNet); ``layers/gst_layers.py:6-168`` (GST,
ReferenceEncoder, StyleTokenLayer, MultiHeadAttention); ``layers/common_layers.py:55-83`` (Prenet,
LinearBN) and the ``Attention`` of ``oracle/tacotron2_torch.py``.

Pinned by tests/test_oracle_torch.py against tests/golden/gst_*.npz / taco_*.npz (the reference's own
outputs).
"""
from __future__ import annotations

from types import SimpleNamespace

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from .tacotron2_torch import _Attention, _t


class _LinearLayer(nn.Module):
    """``Linear`` / ``LinearBN`` of the Prenet: linear_layer [+ bn]."""

    def __init__(self, fin, fout, bn):
        super().__init__()
        self.linear_layer = nn.Linear(fin, fout)
        if bn:
            self.bn = nn.BatchNorm1d(fout)

    def forward(self, x):
        y = self.linear_layer(x)
        return self.bn(y) if hasattr(self, "bn") else y


class _Prenet(nn.Module):
    def __init__(self, fin, bn):
        super().__init__()
        self.layers = nn.ModuleList([_LinearLayer(fin, 256, bn), _LinearLayer(256, 128, bn)])

    def forward(self, x):
        for layer in self.layers:
            x = F.dropout(F.relu(layer(x)), p=0.5, training=False)
        return x


class _BNConv(nn.Module):
    """BatchNormConv1d: constant pad -> Conv1d (no bias) -> BatchNorm1d(eps 1e-3) -> activation."""

    def __init__(self, cin, cout, k, pad, act):
        super().__init__()
        self.padder = nn.ConstantPad1d(pad, 0)
        self.conv1d = nn.Conv1d(cin, cout, k, bias=False)
        self.bn = nn.BatchNorm1d(cout, eps=1e-3)
        self.activation = act

    def forward(self, x):
        x = self.bn(self.conv1d(self.padder(x)))
        return self.activation(x) if self.activation is not None else x


class _Highway(nn.Module):
    def __init__(self, n):
        super().__init__()
        self.H = nn.Linear(n, n)
        self.T = nn.Linear(n, n)

    def forward(self, x):
        t = torch.sigmoid(self.T(x))
        return torch.relu(self.H(x)) * t + x * (1.0 - t)


class _CBHG(nn.Module):
    def __init__(self, fin, K, projections):
        super().__init__()
        self.fin = fin
        relu = nn.ReLU()
        self.conv1d_banks = nn.ModuleList([_BNConv(fin, 128, k, [(k - 1) // 2, k // 2], relu) for k in range(1, K + 1)])
        self.max_pool1d = nn.Sequential(nn.ConstantPad1d([0, 1], value=0), nn.MaxPool1d(kernel_size=2, stride=1))
        ins = [K * 128] + projections[:-1]
        acts = [relu] * (len(projections) - 1) + [None]
        self.conv1d_projections = nn.ModuleList([_BNConv(i, o, 3, [1, 1], a) for i, o, a in zip(ins, projections, acts)])
        if projections[-1] != 128:
            self.pre_highway = nn.Linear(projections[-1], 128, bias=False)
        self.highways = nn.ModuleList([_Highway(128) for _ in range(4)])
        self.gru = nn.GRU(128, 128, 1, batch_first=True, bidirectional=True)

    def forward(self, inputs):
        x = inputs.transpose(1, 2) if inputs.size(-1) == self.fin else inputs
        x = torch.cat([conv(x) for conv in self.conv1d_banks], dim=1)
        x = self.max_pool1d(x)
        for conv in self.conv1d_projections:
            x = conv(x)
        x = x.transpose(1, 2)
        x += inputs
        if hasattr(self, "pre_highway"):
            x = self.pre_highway(x)
        for hw in self.highways:
            x = hw(x)
        self.gru.flatten_parameters()
        return self.gru(x)[0]


class _Holder(nn.Module):
    """A named level of the module tree (the reference's EncoderCBHG / PostCBHG wrappers)."""

    def __init__(self, **mods):
        super().__init__()
        for k, v in mods.items():
            setattr(self, k, v)


class _RefEncoder(nn.Module):
    def __init__(self):
        super().__init__()
        f = [1, 32, 32, 64, 64, 128, 128]
        self.convs = nn.ModuleList([nn.Conv2d(f[i], f[i + 1], 3, 2, 1) for i in range(6)])
        self.bns = nn.ModuleList([nn.BatchNorm2d(c) for c in f[1:]])
        h = 80
        for _ in range(6):
            h = (h - 3 + 2) // 2 + 1
        self.recurrence = nn.GRU(128 * h, 128, batch_first=True)

    def forward(self, mel):
        B = mel.size(0)
        x = mel.view(B, 1, -1, 80)
        for conv, bn in zip(self.convs, self.bns):
            x = F.relu(bn(conv(x)))
        x = x.transpose(1, 2)
        x = x.contiguous().view(B, x.size(1), -1)
        self.recurrence.flatten_parameters()
        return self.recurrence(x)[1].squeeze(0)


class _MHA(nn.Module):
    def __init__(self):
        super().__init__()
        self.W_query = nn.Linear(128, 256, bias=False)
        self.W_key = nn.Linear(64, 256, bias=False)
        self.W_value = nn.Linear(64, 256, bias=False)

    def forward(self, query, key):
        q = torch.stack(torch.split(self.W_query(query), 64, dim=2), 0)
        k = torch.stack(torch.split(self.W_key(key), 64, dim=2), 0)
        v = torch.stack(torch.split(self.W_value(key), 64, dim=2), 0)
        s = F.softmax(torch.matmul(q, k.transpose(2, 3)) / 8.0, dim=3)
        return torch.cat(torch.split(torch.matmul(s, v), 1, dim=0), dim=3).squeeze(0)


class _StyleTokens(nn.Module):
    def __init__(self):
        super().__init__()
        self.style_tokens = nn.Parameter(torch.zeros(10, 64))
        self.attention = _MHA()

    def forward(self, enc):
        tokens = torch.tanh(self.style_tokens).unsqueeze(0).expand(enc.size(0), -1, -1)
        return self.attention(enc.unsqueeze(1), tokens)


class _StopNet(nn.Module):
    def __init__(self, fin):
        super().__init__()
        self.dropout = nn.Dropout(0.1)
        self.linear = nn.Linear(fin, 1)

    def forward(self, x):
        return self.linear(self.dropout(x))


class _Decoder(nn.Module):
    def __init__(self, sd, r, memory_size, bn, flags):
        super().__init__()
        self.r = r
        self.memory_size = memory_size if memory_size > 0 else r
        self.prenet = _Prenet(80 * self.memory_size, bn)
        self.attention_rnn = nn.GRUCell(256 + 128, 256)
        self.attention_layer = _Attention(sd, flags)
        self.project_to_decoder_in = nn.Linear(512, 256)
        self.decoder_rnns = nn.ModuleList([nn.GRUCell(256, 256) for _ in range(2)])
        self.proj_to_mel = nn.Linear(256, 80 * r)
        self.attention_rnn_init = nn.Embedding(1, 256)
        self.memory_init = nn.Embedding(1, self.memory_size * 80)
        self.decoder_rnn_inits = nn.Embedding(2, 256)
        self.stopnet = _StopNet(256 + 80 * r)
        self.max_decoder_steps = 500

    def inference(self, inputs):
        B, L = inputs.size(0), inputs.size(1)
        zero = inputs.new_zeros(B).long()
        memory = self.memory_init(zero)
        h_att = self.attention_rnn_init(zero)
        h_dec = [self.decoder_rnn_inits(inputs.new_tensor([i] * B).long()) for i in range(2)]
        ctx = inputs.new_zeros(B, inputs.size(2))
        P = self.attention_layer.inputs_layer(inputs)
        self.attention_layer.init_states(inputs)
        outs, aligns, stops, t = [], [], [], 0
        while True:
            if t > 0:  # memory queue (layers/tacotron.py:396-404)
                memory = torch.cat([memory[:, self.r * 80:].clone(), outs[-1]], dim=-1)
            h_att = self.attention_rnn(torch.cat((self.prenet(memory), ctx), -1), h_att)
            ctx = self.attention_layer(h_att, inputs, P)
            d = self.project_to_decoder_in(torch.cat((h_att, ctx), -1))
            for i, rnn in enumerate(self.decoder_rnns):
                h_dec[i] = rnn(d, h_dec[i])
                d = h_dec[i] + d
            out = torch.sigmoid(self.proj_to_mel(d))
            stop = torch.sigmoid(self.stopnet(torch.cat([d, out], -1).detach()).data)
            att = self.attention_layer.attention_weights
            outs.append(out)
            aligns.append(att)
            stops.append(stop)
            t += 1
            if t > L / 4 and (stop > 0.6 or att[:, -1].item() > 0.6):
                break
            elif t > self.max_decoder_steps:
                break
        return (torch.stack(outs).transpose(0, 1).contiguous(), torch.stack(aligns).transpose(0, 1),
                torch.stack(stops).transpose(0, 1).squeeze(-1))


class TacotronTorchCPU(nn.Module):
    """Tacotron / TacotronGST (``gst``) from a reference-keyed state dict (numpy or torch); flags as
    ``TacotronOracle``."""

    def __init__(self, sd, r=5, memory_size=5, attn_norm="sigmoid", forward_attn=True, trans_agent=False,
                 forward_attn_mask=False, location_attn=False, attn_win=False, max_decoder_steps=500,
                 prenet_type="original", model="TacotronGST", **_):
        super().__init__()
        self.embedding = nn.Embedding(_t(sd["embedding.weight"]).shape[0], 256)
        if "speaker_embedding.weight" in sd:
            self.speaker_embedding = nn.Embedding(_t(sd["speaker_embedding.weight"]).shape[0], 256)
        self.encoder = _Holder(prenet=_Prenet(256, False), cbhg=_Holder(cbhg=_CBHG(128, 16, [128, 128])))
        if model == "TacotronGST":
            self.gst = _Holder(encoder=_RefEncoder(), style_token_layer=_StyleTokens())
        flags = SimpleNamespace(attn_norm=attn_norm, forward_attn=forward_attn, trans_agent=trans_agent,
                                forward_attn_mask=forward_attn_mask, location_attn=location_attn, attn_win=attn_win)
        self.decoder = _Decoder(sd, r, memory_size, prenet_type == "bn", flags)
        self.decoder.max_decoder_steps = max_decoder_steps
        self.postnet = _Holder(cbhg=_CBHG(80, 8, [256, 80]))
        self.last_linear = nn.Sequential(nn.Linear(256, _t(sd["last_linear.0.weight"]).shape[0]), nn.Sigmoid())
        self.load_state_dict({k: _t(v) for k, v in sd.items()}, strict=True)
        self.eval()

    def encode(self, ids, speaker_id=None, style_mel=None):
        x = self.embedding(torch.as_tensor(np.asarray(ids), dtype=torch.long)[None])
        out = self.encoder.cbhg.cbhg(self.encoder.prenet(x))
        if speaker_id is not None and hasattr(self, "speaker_embedding"):
            e = self.speaker_embedding(torch.as_tensor([speaker_id])).unsqueeze(1)
            out = out + e.expand(out.size(0), out.size(1), -1)
        if style_mel is not None and hasattr(self, "gst"):
            g = self.gst.style_token_layer(self.gst.encoder(torch.as_tensor(np.asarray(style_mel)).float()[None]))
            out = out + g.expand(-1, out.size(1), -1)
        return out

    @torch.no_grad()
    def inference(self, ids, speaker_id=None, style_mel=None):
        enc = self.encode(ids, speaker_id, style_mel)
        mel, align, stop = self.decoder.inference(enc)
        mel = mel.view(1, -1, 80)
        lin = self.last_linear(self.postnet.cbhg(mel))
        return dict(enc=enc[0].numpy(), mel=mel[0].numpy(), linear=lin[0].numpy(), stop=stop[0].numpy(),
                    align=align[0].numpy())
