"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py) — Tacotron2 inference restated in numpy.

Follows the reference op for op, batch-1 semantics (the reference decoder is effectively
batch-1: its stop rule reads item 0, ``layers/tacotron2.py:268``).  A batch is checked
sentence by sentence: ``infer_batch`` runs each sentence alone at its own length, which is
the per-sentence semantics the HIP path implements for padded batches.

Pinned against ``tests/golden/t2_*.npz`` (the reference itself, run on the same weights).
"""
from __future__ import annotations

import numpy as np


def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


class Tacotron2Oracle:
    """``sd``: reference-keyed state dict of numpy arrays; ``cfg``: model flags as in
    ``utils/generic_utils.py:275-288`` (attn_norm, forward_attn, trans_agent,
    forward_attn_mask, location_attn, attn_win, r)."""

    def __init__(self, sd, r=1, attn_norm="sigmoid", forward_attn=True, trans_agent=False,
                 forward_attn_mask=True, location_attn=False, attn_win=False,
                 max_decoder_steps=1000, dtype=np.float64):
        self.dt = dtype
        self.w = {k: np.asarray(v).astype(dtype) if np.asarray(v).dtype.kind == "f" else v
                  for k, v in sd.items()}
        self.r = r
        self.attn_norm = attn_norm
        self.forward_attn = forward_attn
        self.trans_agent = trans_agent
        self.forward_attn_mask = forward_attn_mask
        self.location_attn = location_attn
        self.attn_win = attn_win
        self.max_decoder_steps = max_decoder_steps

    # ------------------------------------------------------------------ building blocks
    def _conv_bn(self, prefix, x, act):
        """ConvBNBlock eval (layers/tacotron2.py:9-27): conv1d k, pad (k-1)/2 -> BN -> act.
        x: [Cin, T] -> [Cout, T]."""
        W = self.w[prefix + ".net.0.weight"]
        b = self.w[prefix + ".net.0.bias"]
        k = W.shape[2]
        p = (k - 1) // 2
        T = x.shape[1]
        xp = np.pad(x, ((0, 0), (p, p)))
        y = np.zeros((W.shape[0], T), dtype=self.dt)
        for j in range(k):
            y += W[:, :, j] @ xp[:, j:j + T]
        y += b[:, None]
        g = self.w[prefix + ".net.1.weight"]
        be = self.w[prefix + ".net.1.bias"]
        mu = self.w[prefix + ".net.1.running_mean"]
        var = self.w[prefix + ".net.1.running_var"]
        y = (y - mu[:, None]) / np.sqrt(var[:, None] + 1e-5) * g[:, None] + be[:, None]
        if act == "relu":
            y = np.maximum(y, 0)
        elif act == "tanh":
            y = np.tanh(y)
        return y

    @staticmethod
    def _lstm_cell(x, h, c, Wih, Whh, bih, bhh):
        g = Wih @ x + bih + Whh @ h + bhh
        H = h.shape[0]
        i, f, gg, o = g[:H], g[H:2 * H], g[2 * H:3 * H], g[3 * H:]
        c2 = _sig(f) * c + _sig(i) * np.tanh(gg)
        return _sig(o) * np.tanh(c2), c2

    # ------------------------------------------------------------------ encoder
    def encoder(self, ids, speaker_id=None, state=None, return_state=False):
        """Tacotron2.inference embedding + Encoder.inference (models/tacotron2.py:63-66,
        layers/tacotron2.py:78-83).  ids [L] -> [L, 512].  ``state`` = (h [2,256], c [2,256]) is the
        BiLSTM's initial state (Encoder.inference_truncated, :85-93; None = zeros)."""
        x = self.w["embedding.weight"][ids].T  # [512, L]
        for i in range(3):
            x = self._conv_bn(f"encoder.convolutions.{i}", x, "relu")
        x = x.T  # [L, 512]
        L = x.shape[0]
        out = np.zeros((L, 512), dtype=self.dt)
        hN = np.zeros((2, 256), self.dt)
        cN = np.zeros((2, 256), self.dt)
        for d, sfx, order in ((0, "", range(L)), (1, "_reverse", range(L - 1, -1, -1))):
            h = np.zeros(256, self.dt) if state is None else state[0][d].astype(self.dt)
            c = np.zeros(256, self.dt) if state is None else state[1][d].astype(self.dt)
            p = [self.w[f"encoder.lstm.{n}_l0{sfx}"] for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
            for t in order:
                h, c = self._lstm_cell(x[t], h, c, *p)
                out[t, d * 256:(d + 1) * 256] = h
            hN[d], cN[d] = h, c
        if speaker_id is not None and "speaker_embedding.weight" in self.w:
            out = out + self.w["speaker_embedding.weight"][speaker_id][None, :]
        return (out, (hN, cN)) if return_state else out

    # ------------------------------------------------------------------ decoder
    def _prenet_layer(self, i, x):
        """Prenet layer i without its ReLU: Linear(bias=False) (layers/tacotron2.py:114), then for
        prenet_type "bn" BatchNorm1d in eval mode (common_layers.py:45-52; running statistics,
        eps 1e-5), present when the state dict holds its keys."""
        p = f"decoder.prenet.layers.{i}."
        y = self.w[p + "linear_layer.weight"] @ x
        if p + "bn.weight" in self.w:
            y = ((y - self.w[p + "bn.running_mean"]) / np.sqrt(self.w[p + "bn.running_var"] + 1e-5) *
                 self.w[p + "bn.weight"] + self.w[p + "bn.bias"])
        return y

    def decoder(self, memory_in, carry=None, return_carry=False, teacher=None):
        """Decoder.inference (layers/tacotron2.py:249-285) for one sentence; with ``teacher`` ([T, 80]
        frames) Decoder.forward (:227-247) instead: step t decodes from the go frame (t = 0) or teacher
        row t-1 (_reshape_memory: r frames per row), exactly T/r steps, no stop rule, and the stop
        outputs are the stopnet logits (forward applies no sigmoid).
        memory_in [L, 512] -> mel [T*r, 80], stop [T], align [T, L].  ``carry`` = (h_att, c_att,
        h_dec, c_dec, ctx, memory) continues from a previous call (Decoder.inference_truncated,
        :287-328: RNN states, context and the last mel frame kept; attention restarts)."""
        w = self.w
        dt = self.dt
        inputs = memory_in.astype(dt)
        L = inputs.shape[0]
        P = inputs @ w["decoder.attention_layer.inputs_layer.linear_layer.weight"].T  # [L,128]
        # _init_states (:157-177) and Attention.init_states (common_layers.py:139-161)
        h_att = w["decoder.attention_rnn_init.weight"][0].copy()
        c_att = np.zeros(1024, dt)
        h_dec = w["decoder.decoder_rnn_inits.weight"][0].copy()
        c_dec = np.zeros(1024, dt)
        ctx = np.zeros(512, dt)
        att_w = np.zeros(L, dt)
        att_cum = np.zeros(L, dt)
        alpha = np.concatenate([[1.0], np.zeros(L - 1) + 1e-7]).astype(dt)
        # float32 reference: torch.zeros + 1e-7 is rounded to float32
        alpha = alpha.astype(np.float32).astype(dt)
        u = 0.5
        win_idx = -1
        memory = w["decoder.go_frame_init.weight"][0].copy()
        if carry is not None:
            h_att, c_att, h_dec, c_dec, ctx, memory = [np.array(v, dtype=dt) for v in carry]
        outs, stops, aligns = [], [], []
        if teacher is not None:
            teacher = np.asarray(teacher, dtype=dt).reshape(-1, 80 * self.r)  # [T/r, 80 r]
        flag1 = False
        stop_count = 0
        t = 0
        while True:
            # Prenet (common_layers.py:77-83), eval: no dropout; prenet_type "bn": LinearBN (:28-52)
            x = np.maximum(self._prenet_layer(0, memory), 0)
            x = np.maximum(self._prenet_layer(1, x), 0)
            # decode() (:194-225)
            h_att, c_att = self._lstm_cell(np.concatenate([x, ctx]), h_att, c_att,
                                           w["decoder.attention_rnn.weight_ih"], w["decoder.attention_rnn.weight_hh"],
                                           w["decoder.attention_rnn.bias_ih"], w["decoder.attention_rnn.bias_hh"])
            # Attention.forward (common_layers.py:225-256)
            pq = w["decoder.attention_layer.query_layer.linear_layer.weight"] @ h_att
            pre = pq[None, :] + P
            if self.location_attn:
                cat = np.stack([att_w, att_cum])  # [2, L]
                cw = w["decoder.attention_layer.location_layer.location_conv.weight"]  # [32,2,31]
                pad = (cw.shape[2] - 1) // 2
                catp = np.pad(cat, ((0, 0), (pad, pad)))
                conv = np.zeros((cw.shape[0], L), dt)
                for j in range(cw.shape[2]):
                    conv += cw[:, :, j] @ catp[:, j:j + L]
                loc = conv.T @ w["decoder.attention_layer.location_layer.location_dense.linear_layer.weight"].T
                pre = pq[None, :] + loc + P
            e = np.tanh(pre) @ w["decoder.attention_layer.v.linear_layer.weight"][0] + \
                w["decoder.attention_layer.v.linear_layer.bias"][0]
            if self.attn_win:  # apply_windowing (common_layers.py:184-197)
                back, front = win_idx - 2, win_idx + 6
                if back > 0:
                    e[:back] = -np.inf
                if front < L:
                    e[front:] = -np.inf
                if win_idx == -1:
                    e[0] = e.max()
                win_idx = int(np.argmax(e))
            if self.attn_norm == "softmax":
                ex = np.exp(e - e.max())
                align = ex / ex.sum()
            elif self.attn_norm == "sigmoid":
                s = _sig(e)
                align = s / s.sum()
            else:
                raise RuntimeError("Unknown value for attention norm type")
            if self.location_attn:
                att_cum = att_cum + align
            if self.forward_attn:  # apply_forward_attention (common_layers.py:199-223)
                prev = np.concatenate([[0.0], alpha[:-1]]).astype(dt)
                a = ((1 - u) * alpha + u * prev + 1e-8) * align
                if self.forward_attn_mask:
                    n = int(np.argmax(prev))
                    val = a.max()
                    # Python slice semantics of common_layers.py:211-213, including the
                    # negative-index wrap when n < 2 (n=0: ':-1' zeroes all but the last
                    # element, and n-2 writes L-2; n=1: n-2 writes L-1).
                    a[n + 3:] = 0
                    if n >= 1:
                        a[:n - 1] = 0
                    else:
                        a[:L - 1] = 0
                    a[(n - 2) % L] = 0.01 * val
                alpha = a / a.sum()
                ctx = alpha @ inputs
                if self.trans_agent:
                    ta = w["decoder.attention_layer.ta.weight"][0] @ np.concatenate([ctx, h_att]) + \
                        w["decoder.attention_layer.ta.bias"][0]
                    u = _sig(ta)
                att_w = alpha
            else:
                ctx = align @ inputs
                att_w = align
            h_dec, c_dec = self._lstm_cell(np.concatenate([h_att, ctx]), h_dec, c_dec,
                                           w["decoder.decoder_rnn.weight_ih"], w["decoder.decoder_rnn.weight_hh"],
                                           w["decoder.decoder_rnn.bias_ih"], w["decoder.decoder_rnn.bias_hh"])
            mel = w["decoder.linear_projection.linear_layer.weight"] @ np.concatenate([h_dec, ctx]) + \
                w["decoder.linear_projection.linear_layer.bias"]
            st = w["decoder.stopnet.1.linear_layer.weight"][0] @ np.concatenate([h_dec, mel]) + \
                w["decoder.stopnet.1.linear_layer.bias"][0]
            outs.append(mel)
            stops.append(st if teacher is not None else _sig(st))
            aligns.append(att_w.copy())
            if teacher is not None:
                if len(outs) == teacher.shape[0]:
                    break
                memory = teacher[t]
                t += 1
                continue
            # stop rule (:267-277); stop_flags[0] starts True and is never cleared
            flag1 = flag1 or (att_w[-2:].sum() > 0.8 and t > L)
            flag2 = t > 2 * L
            if flag1 and flag2:
                stop_count += 1
                if stop_count > 20:
                    break
            elif len(outs) == self.max_decoder_steps:
                break
            memory = mel
            t += 1
        mel = np.stack(outs).reshape(-1, 80)  # [T*r, 80]
        if return_carry:
            return mel, np.array(stops), np.stack(aligns), (h_att, c_att, h_dec, c_dec, ctx, outs[-1])
        return mel, np.array(stops), np.stack(aligns)

    def postnet(self, mel):
        """Postnet (layers/tacotron2.py:30-45) + residual (models/tacotron2.py:69-70).
        mel [T, 80] -> mel_post [T, 80]."""
        x = mel.T.astype(self.dt)
        for i in range(5):
            x = self._conv_bn(f"postnet.convolutions.{i}", x, "tanh" if i < 4 else None)
        return mel + x.T

    def inference(self, ids, speaker_id=None):
        """Tacotron2.inference (models/tacotron2.py:62-73) for one sentence."""
        enc = self.encoder(np.asarray(ids), speaker_id)
        mel, stop, align = self.decoder(enc)
        return dict(enc=enc, mel=mel, mel_post=self.postnet(mel), stop=stop, align=align)

    def inference_truncated(self, ids_seq):
        """Tacotron2.inference_truncated (models/tacotron2.py:75-89) over consecutive texts: the
        encoder BiLSTM state and the decoder carry pass from one call to the next."""
        enc_state, carry, res = None, None, []
        for ids in ids_seq:
            enc, enc_state = self.encoder(np.asarray(ids), None, enc_state, return_state=True)
            mel, stop, align, carry = self.decoder(enc, carry, return_carry=True)
            res.append(dict(enc=enc, mel=mel, mel_post=self.postnet(mel), stop=stop, align=align))
        return res

    def forward(self, ids, teacher, speaker_id=None):
        """Tacotron2.forward (models/tacotron2.py:47-60) in eval mode for one sentence: encoder at its
        length, teacher-forced decoder, postnet + residual."""
        enc = self.encoder(np.asarray(ids), speaker_id)
        mel, stop, align = self.decoder(enc, teacher=teacher)
        return dict(enc=enc, mel=mel, mel_post=self.postnet(mel), stop=stop, align=align)

    def infer_batch(self, ids_list):
        return [self.inference(ids) for ids in ids_list]
