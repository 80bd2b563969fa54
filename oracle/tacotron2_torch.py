"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py) — Tacotron2 inference restated on torch CPU.

The CPU *baseline* leg of ``bench.py`` (and tools/cpu_port_vs_reference.py).  Same algorithm as
``tacotron2_oracle.Tacotron2Oracle`` (which stays the parity checker), restated as a tree of torch
``nn`` modules that call the same CPU kernels in the same per-step order as the reference — the
LSTM cells as ``nn.LSTMCell``, every linear layer behind a one-level wrapper module as the
reference's ``Linear``, the eval-mode dropouts as the no-op calls the reference makes, the forward
attention's clones and its per-sentence mask loop, the stop rule's tensor comparisons — so that
the host time of a sentence matches the reference's own on the same cores (BASELINE.md section
3.2).  Round 5: a functional restatement (``F.linear`` on bare tensors) ran the same kernels but
0.68x the reference's time at 8 threads (profiles/cpu_port_vs_reference_r04.json): the per-step
module and dispatch overhead between ops is part of the reference's CPU path, so it is kept.
Nothing here is shipped: the product path never imports ``oracle/``.

Reference lines followed: ``models/tacotron2.py:62-73`` (inference), ``layers/tacotron2.py:9-27``
(ConvBNBlock), ``:30-45`` (Postnet), ``:78-83`` (Encoder.inference), ``:157-177`` (_init_states),
``:194-225`` (decode), ``:249-285`` (Decoder.inference + stop rule), ``layers/common_layers.py:8-25``
(Linear), ``:77-83`` (Prenet), ``:86-104`` (LocationLayer), ``:139-161`` (attention init),
``:163-182`` (energies), ``:184-197`` (windowing), ``:199-223`` (forward attention), ``:225-256``
(Attention.forward).

Pinned by tests/test_oracle_torch.py against tests/golden/t2_*.npz (the reference's own outputs).
"""
from __future__ import annotations

from types import SimpleNamespace

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn


def _t(v):
    t = torch.as_tensor(np.asarray(v))
    return t.float() if t.is_floating_point() else t


class _Wrapped(nn.Module):
    """One extra module level around ``nn.Linear`` (the reference's ``Linear`` wrapper)."""

    def __init__(self, w, b=None):
        super().__init__()
        self.linear_layer = nn.Linear(w.shape[1], w.shape[0], bias=b is not None)
        with torch.no_grad():
            self.linear_layer.weight.copy_(w)
            if b is not None:
                self.linear_layer.bias.copy_(b)

    def forward(self, x):
        return self.linear_layer(x)


class _ConvBN(nn.Module):
    """ConvBNBlock eval: Conv1d (same padding) -> BatchNorm1d -> activation -> Dropout (no-op)."""

    def __init__(self, sd, prefix, act):
        super().__init__()
        W = _t(sd[prefix + ".net.0.weight"])
        self.conv = nn.Conv1d(W.shape[1], W.shape[0], W.shape[2], padding=(W.shape[2] - 1) // 2)
        self.bn = nn.BatchNorm1d(W.shape[0])
        with torch.no_grad():
            self.conv.weight.copy_(W)
            self.conv.bias.copy_(_t(sd[prefix + ".net.0.bias"]))
            for k in ("weight", "bias", "running_mean", "running_var"):
                getattr(self.bn, k).copy_(_t(sd[f"{prefix}.net.1.{k}"]))
        self.act = {"relu": nn.ReLU(), "tanh": nn.Tanh()}.get(act, nn.Identity())
        self.drop = nn.Dropout(0.5)

    def forward(self, x):
        return self.drop(self.act(self.bn(self.conv(x))))


def _cell(sd, name):
    p = [_t(sd[f"decoder.{name}.{k}"]) for k in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
    c = nn.LSTMCell(p[0].shape[1], p[1].shape[1])
    with torch.no_grad():
        for k, v in zip(("weight_ih", "weight_hh", "bias_ih", "bias_hh"), p):
            getattr(c, k).copy_(v)
    return c


def _table(sd, key):
    W = _t(sd[key])
    e = nn.Embedding(W.shape[0], W.shape[1])
    with torch.no_grad():
        e.weight.copy_(W)
    return e


class _Attention(nn.Module):
    def __init__(self, sd, owner):
        super().__init__()
        a = "decoder.attention_layer."
        self.o = owner
        self.query_layer = _Wrapped(_t(sd[a + "query_layer.linear_layer.weight"]))
        self.inputs_layer = _Wrapped(_t(sd[a + "inputs_layer.linear_layer.weight"]))
        self.v = _Wrapped(_t(sd[a + "v.linear_layer.weight"]), _t(sd[a + "v.linear_layer.bias"]))
        if owner.location_attn:
            cw = _t(sd[a + "location_layer.location_conv.weight"])
            self.location_layer = nn.Module()
            self.location_layer.location_conv = nn.Conv1d(2, cw.shape[0], cw.shape[2], padding=(cw.shape[2] - 1) // 2,
                                                          bias=False)
            with torch.no_grad():
                self.location_layer.location_conv.weight.copy_(cw)
            self.location_layer.location_dense = _Wrapped(
                _t(sd[a + "location_layer.location_dense.linear_layer.weight"]))
        if owner.trans_agent:
            self.ta = nn.Linear(_t(sd[a + "ta.weight"]).shape[1], 1)
            with torch.no_grad():
                self.ta.weight.copy_(_t(sd[a + "ta.weight"]))
                self.ta.bias.copy_(_t(sd[a + "ta.bias"]))

    def init_states(self, inputs):
        B, T = inputs.shape[0], inputs.shape[1]
        self.attention_weights = inputs.new_zeros(B, T)
        if self.o.location_attn:
            self.attention_weights_cum = inputs.new_zeros(B, T)
        if self.o.forward_attn:
            self.alpha = torch.cat([torch.ones(B, 1), torch.zeros(B, T)[:, :-1] + 1e-7], 1)
            self.u = 0.5 * torch.ones(B, 1)
        self.win_idx = -1

    def forward(self, query, inputs, processed_inputs):
        o = self.o
        pq = self.query_layer(query.unsqueeze(1))
        if o.location_attn:
            cat = torch.cat((self.attention_weights.unsqueeze(1), self.attention_weights_cum.unsqueeze(1)), 1)
            ll = self.location_layer
            loc = ll.location_dense(ll.location_conv(cat).transpose(1, 2))
            energies = self.v(torch.tanh(pq + loc + processed_inputs)).squeeze(-1)
        else:
            energies = self.v(torch.tanh(pq + processed_inputs)).squeeze(-1)
        if o.attn_win:  # eval windowing
            back, front = self.win_idx - 2, self.win_idx + 6
            if back > 0:
                energies[:, :back] = -float("inf")
            if front < inputs.shape[1]:
                energies[:, front:] = -float("inf")
            if self.win_idx == -1:
                energies[:, 0] = energies.max()
            self.win_idx = torch.argmax(energies, 1).long()[0].item()
        if o.attn_norm == "softmax":
            align = torch.softmax(energies, dim=-1)
        elif o.attn_norm == "sigmoid":
            align = torch.sigmoid(energies) / torch.sigmoid(energies).sum(dim=1).unsqueeze(1)
        else:
            raise RuntimeError("Unknown value for attention norm type")
        if o.location_attn:
            self.attention_weights_cum += align
        if o.forward_attn:
            prev = F.pad(self.alpha[:, :-1].clone(), (1, 0, 0, 0)).to(inputs.device)
            a = (((1 - self.u) * self.alpha.clone().to(inputs.device) + self.u * prev) + 1e-8) * align
            if o.forward_attn_mask:
                _, n = prev.max(1)
                val, _ = a.max(1)
                for b in range(align.shape[0]):
                    a[b, n[b] + 3:] = 0
                    a[b, :(n[b] - 1)] = 0  # Python slicing: n = 0 reads ':-1'
                    a[b, (n[b] - 2)] = 0.01 * val[b]  # negative index wraps as in the reference
            self.alpha = a / a.sum(dim=1).unsqueeze(1)
            ctx = torch.bmm(self.alpha.unsqueeze(1), inputs).squeeze(1)
            if o.trans_agent:
                self.u = torch.sigmoid(self.ta(torch.cat([ctx, query], dim=-1)))
            self.attention_weights = self.alpha
        else:
            ctx = torch.bmm(align.unsqueeze(1), inputs).squeeze(1)
            self.attention_weights = align
        return ctx


class Tacotron2TorchCPU(nn.Module):
    """``sd``: reference-keyed state dict (numpy or torch); flags as ``Tacotron2Oracle``."""

    def __init__(self, sd, r=1, attn_norm="sigmoid", forward_attn=True, trans_agent=False,
                 forward_attn_mask=True, location_attn=False, attn_win=False, max_decoder_steps=1000):
        super().__init__()
        self.r = r
        self.attn_norm = attn_norm
        self.forward_attn = forward_attn
        self.trans_agent = trans_agent
        self.forward_attn_mask = forward_attn_mask
        self.location_attn = location_attn
        self.attn_win = attn_win
        self.max_decoder_steps = max_decoder_steps
        self.embedding = _table(sd, "embedding.weight")
        self.speaker_embedding = _table(sd, "speaker_embedding.weight") if "speaker_embedding.weight" in sd else None
        self.enc_convs = nn.ModuleList([_ConvBN(sd, f"encoder.convolutions.{i}", "relu") for i in range(3)])
        lstm_p = [_t(sd[f"encoder.lstm.{n}_l0{s}"]) for s in ("", "_reverse")
                  for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
        self.lstm = nn.LSTM(lstm_p[0].shape[1], lstm_p[1].shape[1], 1, batch_first=True, bidirectional=True)
        with torch.no_grad():
            for p, v in zip(self.lstm._flat_weights, lstm_p):
                p.copy_(v)
        self.post_convs = nn.ModuleList([_ConvBN(sd, f"postnet.convolutions.{i}", "tanh" if i < 4 else None)
                                         for i in range(5)])
        # decoder
        self.prenet = nn.ModuleList([_Wrapped(_t(sd[f"decoder.prenet.layers.{i}.linear_layer.weight"]))
                                     for i in range(2)])
        self.prenet_bn = None
        if "decoder.prenet.layers.0.bn.weight" in sd:  # prenet_type "bn": LinearBN (eval BatchNorm1d)
            self.prenet_bn = nn.ModuleList()
            for i in range(2):
                bn = nn.BatchNorm1d(self.prenet[i].linear_layer.out_features)
                with torch.no_grad():
                    for k in ("weight", "bias", "running_mean", "running_var"):
                        getattr(bn, k).copy_(_t(sd[f"decoder.prenet.layers.{i}.bn.{k}"]))
                self.prenet_bn.append(bn)
        self.attention_rnn = _cell(sd, "attention_rnn")
        self.decoder_rnn = _cell(sd, "decoder_rnn")
        self.attention_layer = _Attention(sd, SimpleNamespace(
            attn_norm=attn_norm, forward_attn=forward_attn, trans_agent=trans_agent,
            forward_attn_mask=forward_attn_mask, location_attn=location_attn, attn_win=attn_win))
        self.linear_projection = _Wrapped(_t(sd["decoder.linear_projection.linear_layer.weight"]),
                                          _t(sd["decoder.linear_projection.linear_layer.bias"]))
        self.stopnet = nn.Sequential(nn.Dropout(0.1), _Wrapped(_t(sd["decoder.stopnet.1.linear_layer.weight"]),
                                                               _t(sd["decoder.stopnet.1.linear_layer.bias"])))
        self.go_frame_init = _table(sd, "decoder.go_frame_init.weight")
        self.attention_rnn_init = _table(sd, "decoder.attention_rnn_init.weight")
        self.decoder_rnn_inits = _table(sd, "decoder.decoder_rnn_inits.weight")
        self.eval()

    # ------------------------------------------------------------------ encoder / postnet
    def encoder(self, ids, speaker_id=None):
        """ids [L] -> [1, L, 512]."""
        x = self.embedding(torch.as_tensor(np.asarray(ids), dtype=torch.long)[None]).transpose(1, 2)
        for c in self.enc_convs:
            x = c(x)
        x = x.transpose(1, 2)
        self.lstm.flatten_parameters()
        out, _ = self.lstm(x)
        if speaker_id is not None and self.speaker_embedding is not None:
            out = out + self.speaker_embedding(torch.as_tensor([speaker_id])).unsqueeze(1)
        return out

    def postnet(self, mel):
        """mel [1, T, 80] -> mel + Postnet(mel)."""
        x = mel.transpose(1, 2)
        for c in self.post_convs:
            x = c(x)
        return mel + x.transpose(1, 2)

    # ------------------------------------------------------------------ decoder
    def _prenet(self, x):
        for i, lin in enumerate(self.prenet):
            y = lin(x)
            if self.prenet_bn is not None:
                y = self.prenet_bn[i](y)
            x = F.dropout(F.relu(y), p=0.5, training=False)
        return x

    def decoder(self, inputs):
        """inputs [1, L, 512] -> mel [1, T*r, 80] (frame-major), stop [T], align [T, L]."""
        B, L = inputs.shape[0], inputs.shape[1]
        zero = inputs.new_zeros(B).long()
        memory = self.go_frame_init(zero)
        h_att, c_att = self.attention_rnn_init(zero), inputs.new_zeros(B, 1024)
        h_dec, c_dec = self.decoder_rnn_inits(zero), inputs.new_zeros(B, 1024)
        ctx = inputs.new_zeros(B, inputs.shape[2])
        P = self.attention_layer.inputs_layer(inputs)
        self.attention_layer.init_states(inputs)
        outs, stops, aligns, t = [], [], [], 0
        flags = [True, False, False]
        stop_count = 0
        while True:
            memory = self._prenet(memory)
            h_att, c_att = self.attention_rnn(torch.cat((memory, ctx), -1), (h_att, c_att))
            h_att = F.dropout(h_att, 0.1, False)
            c_att = F.dropout(c_att, 0.1, False)
            ctx = self.attention_layer(h_att, inputs, P)
            h_dec, c_dec = self.decoder_rnn(torch.cat((h_att, ctx), -1), (h_dec, c_dec))
            h_dec = F.dropout(h_dec, 0.1, False)
            c_dec = F.dropout(c_dec, 0.1, False)
            mel = self.linear_projection(torch.cat((h_dec, ctx), dim=1))
            stop = torch.sigmoid(self.stopnet(torch.cat((h_dec, mel), dim=1).detach()).data)
            align = self.attention_layer.attention_weights
            outs.append(mel.squeeze(1))
            stops.append(stop)
            aligns.append(align)
            # stop rule (layers/tacotron2.py:267-277); flags[0] starts True and is never cleared
            flags[0] = flags[0] or stop > 0.5
            flags[1] = flags[1] or (align[0, -2:].sum() > 0.8 and t > L)
            flags[2] = t > L * 2
            if all(flags):
                stop_count += 1
                if stop_count > 20:
                    break
            elif len(outs) == self.max_decoder_steps:
                break
            memory = mel
            t += 1
        mel = torch.stack(outs).transpose(0, 1).contiguous().view(B, -1, 80)
        return mel, torch.stack(stops).transpose(0, 1).reshape(-1), torch.stack(aligns).transpose(0, 1)[0]

    @torch.no_grad()
    def inference(self, ids, speaker_id=None):
        enc = self.encoder(ids, speaker_id)
        mel, stop, align = self.decoder(enc)
        post = self.postnet(mel)
        return dict(enc=enc[0].numpy(), mel=mel[0].numpy(), mel_post=post[0].numpy(), stop=stop.numpy(),
                    align=align.numpy())
