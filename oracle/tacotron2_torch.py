"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py) — Tacotron2 inference restated on torch CPU ops.

The CPU *baseline* leg of ``bench.py`` (and tools/cpu_port_vs_reference.py).  Same algorithm as
``tacotron2_oracle.Tacotron2Oracle`` (which stays the parity checker), restated with the torch CPU
kernels the reference runs on — ``torch.lstm_cell`` (the op behind ``nn.LSTMCell``), ``F.linear``
(addmm / mv), ``F.conv1d`` + ``F.batch_norm`` (eval) — in the reference's per-step op order,
batch dimension 1 kept as the reference keeps it, so that its time on a host equals the
reference's time on the same cores.  Nothing here is shipped: the
product path never imports ``oracle/``.

Reference lines followed: ``models/tacotron2.py:62-73`` (inference), ``layers/tacotron2.py:9-27``
(ConvBNBlock), ``:30-45`` (Postnet), ``:78-83`` (Encoder.inference), ``:157-177`` (_init_states),
``:194-225`` (decode), ``:249-285`` (Decoder.inference + stop rule), ``layers/common_layers.py:77-83``
(Prenet), ``:139-161`` (attention init), ``:163-182`` (energies), ``:184-197`` (windowing),
``:199-223`` (forward attention), ``:225-256`` (Attention.forward).

Pinned by tests/test_oracle_torch.py against tests/golden/t2_*.npz (the reference's own outputs).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


class Tacotron2TorchCPU:
    """``sd``: reference-keyed state dict (numpy or torch); flags as ``Tacotron2Oracle``."""

    def __init__(self, sd, r=1, attn_norm="sigmoid", forward_attn=True, trans_agent=False,
                 forward_attn_mask=True, location_attn=False, attn_win=False, max_decoder_steps=1000):
        self.w = {k: torch.as_tensor(np.asarray(v)) for k, v in sd.items()}
        self.w = {k: (v.float() if v.is_floating_point() else v) for k, v in self.w.items()}
        self.r = r
        self.attn_norm = attn_norm
        self.forward_attn = forward_attn
        self.trans_agent = trans_agent
        self.forward_attn_mask = forward_attn_mask
        self.location_attn = location_attn
        self.attn_win = attn_win
        self.max_decoder_steps = max_decoder_steps
        self._cell = {n: tuple(self.w[f"decoder.{n}.{p}"] for p in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"))
                      for n in ("attention_rnn", "decoder_rnn")}

    # ------------------------------------------------------------------ conv stacks
    def _conv_bn(self, prefix, x, act):
        """ConvBNBlock eval: x [1, Cin, T] -> [1, Cout, T]."""
        w = self.w
        W = w[prefix + ".net.0.weight"]
        y = F.conv1d(x, W, w[prefix + ".net.0.bias"], padding=(W.shape[2] - 1) // 2)
        y = F.batch_norm(y, w[prefix + ".net.1.running_mean"], w[prefix + ".net.1.running_var"],
                         w[prefix + ".net.1.weight"], w[prefix + ".net.1.bias"], False, 0.0, 1e-5)
        if act == "relu":
            return torch.relu(y)
        if act == "tanh":
            return torch.tanh(y)
        return y

    def encoder(self, ids, speaker_id=None):
        """ids [L] -> [1, L, 512]."""
        w = self.w
        x = F.embedding(torch.as_tensor(np.asarray(ids), dtype=torch.long)[None], w["embedding.weight"])
        x = x.transpose(1, 2)
        for i in range(3):
            x = self._conv_bn(f"encoder.convolutions.{i}", x, "relu")
        x = x.transpose(1, 2).contiguous()
        params = [w[f"encoder.lstm.{n}_l0{s}"] for s in ("", "_reverse")
                  for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
        h0 = torch.zeros(2, 1, 256)
        out = torch.lstm(x, (h0, h0), params, True, 1, 0.0, False, True, True)[0]
        if speaker_id is not None and "speaker_embedding.weight" in w:
            out = out + w["speaker_embedding.weight"][speaker_id][None, None, :]
        return out

    # ------------------------------------------------------------------ decoder
    def _energies(self, h_att, P, att_w, att_cum):
        w = self.w
        pq = F.linear(h_att.unsqueeze(1), w["decoder.attention_layer.query_layer.linear_layer.weight"])
        if self.location_attn:
            cat = torch.stack((att_w, att_cum), 1)
            conv = F.conv1d(cat, w["decoder.attention_layer.location_layer.location_conv.weight"], padding=15)
            loc = F.linear(conv.transpose(1, 2),
                           w["decoder.attention_layer.location_layer.location_dense.linear_layer.weight"])
            pre = pq + loc + P
        else:
            pre = pq + P
        e = F.linear(torch.tanh(pre), w["decoder.attention_layer.v.linear_layer.weight"],
                     w["decoder.attention_layer.v.linear_layer.bias"])
        return e.squeeze(-1)

    def decoder(self, inputs):
        """inputs [1, L, 512] -> mel [1, T*r, 80] (frame-major), stop [T], align [T, L]."""
        w = self.w
        L = inputs.shape[1]
        P = F.linear(inputs, w["decoder.attention_layer.inputs_layer.linear_layer.weight"])
        zero = torch.zeros(1, dtype=torch.long)
        h_att = F.embedding(zero, w["decoder.attention_rnn_init.weight"])
        c_att = torch.zeros(1, 1024)
        h_dec = F.embedding(zero, w["decoder.decoder_rnn_inits.weight"])
        c_dec = torch.zeros(1, 1024)
        ctx = torch.zeros(1, 512)
        att_w = torch.zeros(1, L)
        att_cum = torch.zeros(1, L)
        alpha = torch.cat([torch.ones(1, 1), torch.zeros(1, L)[:, :-1] + 1e-7], 1)
        u = 0.5 * torch.ones(1, 1)
        win_idx = -1
        memory = F.embedding(zero, w["decoder.go_frame_init.weight"])
        def prenet_layer(i, x):  # Linear(bias=False), + eval BatchNorm1d for prenet_type "bn" (:28-52)
            p = f"decoder.prenet.layers.{i}."
            y = F.linear(x, w[p + "linear_layer.weight"])
            if p + "bn.weight" in w:
                y = F.batch_norm(y, w[p + "bn.running_mean"], w[p + "bn.running_var"], w[p + "bn.weight"],
                                 w[p + "bn.bias"], False, 0.0, 1e-5)
            return y
        w_mel, b_mel = w["decoder.linear_projection.linear_layer.weight"], w["decoder.linear_projection.linear_layer.bias"]
        w_st, b_st = w["decoder.stopnet.1.linear_layer.weight"], w["decoder.stopnet.1.linear_layer.bias"]
        outs, stops, aligns = [], [], []
        flags = [True, False, False]
        stop_count = 0
        t = 0
        while True:
            x = torch.relu(prenet_layer(1, torch.relu(prenet_layer(0, memory))))
            h_att, c_att = torch.lstm_cell(torch.cat((x, ctx), -1), (h_att, c_att), *self._cell["attention_rnn"])
            e = self._energies(h_att, P, att_w, att_cum)
            if self.attn_win:
                back, front = win_idx - 2, win_idx + 6
                if back > 0:
                    e[:, :back] = -float("inf")
                if front < L:
                    e[:, front:] = -float("inf")
                if win_idx == -1:
                    e[:, 0] = e.max()
                win_idx = int(torch.argmax(e, 1)[0])
            if self.attn_norm == "softmax":
                align = torch.softmax(e, -1)
            elif self.attn_norm == "sigmoid":
                align = torch.sigmoid(e) / torch.sigmoid(e).sum(1).unsqueeze(1)
            else:
                raise RuntimeError("Unknown value for attention norm type")
            if self.location_attn:
                att_cum = att_cum + align
            if self.forward_attn:
                prev = F.pad(alpha[:, :-1], (1, 0))
                a = ((1 - u) * alpha + u * prev + 1e-8) * align
                if self.forward_attn_mask:
                    n = int(prev.argmax(1)[0])
                    val = a.max(1)[0]
                    a[0, n + 3:] = 0
                    a[0, :n - 1] = 0  # Python slice: n = 0 reads ':-1'
                    a[0, n - 2] = 0.01 * val[0]  # negative index wraps as in the reference
                alpha = a / a.sum(1).unsqueeze(1)
                ctx = torch.bmm(alpha.unsqueeze(1), inputs).squeeze(1)
                if self.trans_agent:
                    u = torch.sigmoid(F.linear(torch.cat([ctx, h_att], -1), w["decoder.attention_layer.ta.weight"],
                                               w["decoder.attention_layer.ta.bias"]))
                att_w = alpha
            else:
                ctx = torch.bmm(align.unsqueeze(1), inputs).squeeze(1)
                att_w = align
            h_dec, c_dec = torch.lstm_cell(torch.cat((h_att, ctx), -1), (h_dec, c_dec), *self._cell["decoder_rnn"])
            mel = F.linear(torch.cat((h_dec, ctx), 1), w_mel, b_mel)
            st = torch.sigmoid(F.linear(torch.cat((h_dec, mel), 1), w_st, b_st))
            outs.append(mel)
            stops.append(st)
            aligns.append(att_w)
            # stop rule; flags[0] starts True and is never cleared
            flags[1] = flags[1] or bool(att_w[0, -2:].sum() > 0.8 and t > L)
            flags[2] = t > 2 * L
            if all(flags):
                stop_count += 1
                if stop_count > 20:
                    break
            elif len(outs) == self.max_decoder_steps:
                break
            memory = mel
            t += 1
        mel = torch.stack(outs, 1).reshape(1, -1, 80)
        return mel, torch.cat(stops, 1).reshape(-1), torch.cat(aligns, 0)

    def postnet(self, mel):
        """mel [1, T, 80] -> mel + Postnet(mel)."""
        x = mel.transpose(1, 2)
        for i in range(5):
            x = self._conv_bn(f"postnet.convolutions.{i}", x, "tanh" if i < 4 else None)
        return mel + x.transpose(1, 2)

    @torch.no_grad()
    def inference(self, ids, speaker_id=None):
        enc = self.encoder(ids, speaker_id)
        mel, stop, align = self.decoder(enc)
        post = self.postnet(mel)
        return dict(enc=enc[0].numpy(), mel=mel[0].numpy(), mel_post=post[0].numpy(), stop=stop.numpy(),
                    align=align.numpy())
