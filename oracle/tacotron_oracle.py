"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py) — Tacotron / TacotronGST inference in numpy.

Follows the reference op for op:
  ``TacotronGST.inference`` (models/tacotrongst.py:64-79) / ``Tacotron.inference``
  (models/tacotron.py:59-70): embedding -> ``Encoder`` (Prenet + CBHG, layers/tacotron.py:225-243)
  -> [+ speaker embedding] -> [+ GST(style_mel) (layers/gst_layers.py:6-168)]
  -> ``Decoder.inference`` (layers/tacotron.py:439-470; ``Attention``, layers/common_layers.py:107-256)
  -> ``PostCBHG`` (layers/tacotron.py:246-259) -> ``last_linear`` + sigmoid.
Batch-1 semantics: the reference's stop rule calls ``.item()`` (layers/tacotron.py:465), so the
reference itself only runs one sentence at a time; a batch is checked sentence by sentence.

Pinned against ``tests/golden/gst_*.npz`` / ``taco_*.npz`` (the reference itself, run by
``tests/golden/make_golden.py`` on the same generated weights).
"""
from __future__ import annotations

import numpy as np


def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def _softmax(x):
    e = np.exp(x - x.max())
    return e / e.sum()


class TacotronOracle:
    """``sd``: reference-keyed state dict of numpy arrays (``weights.tacotron_gst_spec`` order)."""

    def __init__(self, sd, r=5, memory_size=5, attn_norm="sigmoid", forward_attn=True, trans_agent=False,
                 forward_attn_mask=False, location_attn=False, attn_win=False, max_decoder_steps=500,
                 dtype=np.float64, **_):
        self.dt = dtype
        self.w = {k: np.asarray(v).astype(dtype) if np.asarray(v).dtype.kind == "f" else v for k, v in sd.items()}
        self.r = r
        self.memory_size = memory_size if memory_size > 0 else r
        self.attn_norm = attn_norm
        self.forward_attn = forward_attn
        self.trans_agent = trans_agent
        self.forward_attn_mask = forward_attn_mask
        self.location_attn = location_attn
        self.attn_win = attn_win
        self.max_decoder_steps = max_decoder_steps

    # ------------------------------------------------------------------ building blocks
    def _bn(self, prefix, y, eps):
        """BatchNorm1d/2d eval over dim 0 of y [C, ...]."""
        shp = (-1,) + (1,) * (y.ndim - 1)
        g, be = self.w[prefix + ".weight"].reshape(shp), self.w[prefix + ".bias"].reshape(shp)
        mu, var = self.w[prefix + ".running_mean"].reshape(shp), self.w[prefix + ".running_var"].reshape(shp)
        return (y - mu) / np.sqrt(var + eps) * g + be

    def _bn_conv(self, prefix, x, k, pad_l, pad_r, act):
        """BatchNormConv1d (layers/tacotron.py:7-66): ConstantPad1d -> Conv1d (no bias) ->
        BatchNorm1d(eps=1e-3) -> activation.  x [Cin, T] -> [Cout, T]."""
        W = self.w[prefix + ".conv1d.weight"]
        T = x.shape[1]
        xp = np.pad(x, ((0, 0), (pad_l, pad_r)))
        y = np.zeros((W.shape[0], T), self.dt)
        for j in range(k):
            y += W[:, :, j] @ xp[:, j:j + T]
        y = self._bn(prefix + ".bn", y, 1e-3)
        return np.maximum(y, 0) if act == "relu" else y

    @staticmethod
    def _gru_cell(x, h, Wih, Whh, bih, bhh):
        """torch GRUCell: r, z, n gate rows; h' = (h - n) * z + n (ATen's GRUCell)."""
        gi = Wih @ x + bih
        gh = Whh @ h + bhh
        H = h.shape[0]
        r = _sig(gi[:H] + gh[:H])
        z = _sig(gi[H:2 * H] + gh[H:2 * H])
        n = np.tanh(gi[2 * H:] + r * gh[2 * H:])
        return (h - n) * z + n

    def _gru_seq(self, prefix, x, sfx="", reverse=False):
        p = [self.w[f"{prefix}.{n}_l0{sfx}"] for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
        T = x.shape[0]
        H = p[1].shape[1]
        h = np.zeros(H, self.dt)
        out = np.zeros((T, H), self.dt)
        for t in (range(T - 1, -1, -1) if reverse else range(T)):
            h = self._gru_cell(x[t], h, *p)
            out[t] = h
        return out

    def _prenet(self, prefix, x):
        """Prenet eval (layers/common_layers.py:77-83): relu(linear) per layer, no dropout; with
        prenet_type "bn" (the decoder's, layers/tacotron.py:283-287) each linear is followed by an
        eval-mode BatchNorm1d (LinearBN, common_layers.py:28-52; eps 1e-5)."""
        for i in range(2):
            p = f"{prefix}.layers.{i}."
            y = x @ self.w[p + "linear_layer.weight"].T + self.w[p + "linear_layer.bias"]
            if p + "bn.weight" in self.w:
                y = ((y - self.w[p + "bn.running_mean"]) / np.sqrt(self.w[p + "bn.running_var"] + 1e-5) *
                     self.w[p + "bn.weight"] + self.w[p + "bn.bias"])
            x = np.maximum(y, 0)
        return x

    def cbhg(self, prefix, x, K, projections):
        """CBHG.forward (layers/tacotron.py:172-206).  x [T, in_features] -> [T, 256]."""
        inputs = x
        xt = x.T
        outs = [self._bn_conv(f"{prefix}.conv1d_banks.{k - 1}", xt, k, (k - 1) // 2, k // 2, "relu")
                for k in range(1, K + 1)]
        y = np.concatenate(outs, 0)
        yp = np.pad(y, ((0, 0), (0, 1)))  # ConstantPad1d([0, 1], 0) + MaxPool1d(2, stride 1)
        y = np.maximum(yp[:, :-1], yp[:, 1:])
        for i in range(len(projections)):
            y = self._bn_conv(f"{prefix}.conv1d_projections.{i}", y, 3, 1, 1,
                              "relu" if i < len(projections) - 1 else None)
        y = y.T + inputs
        if projections[-1] != 128:
            y = y @ self.w[f"{prefix}.pre_highway.weight"].T
        for i in range(4):  # Highway (layers/tacotron.py:69-89)
            hp = f"{prefix}.highways.{i}"
            Hh = np.maximum(y @ self.w[hp + ".H.weight"].T + self.w[hp + ".H.bias"], 0)
            Tt = _sig(y @ self.w[hp + ".T.weight"].T + self.w[hp + ".T.bias"])
            y = Hh * Tt + y * (1.0 - Tt)
        fwd = self._gru_seq(f"{prefix}.gru", y, "")
        bwd = self._gru_seq(f"{prefix}.gru", y, "_reverse", reverse=True)
        return np.concatenate([fwd, bwd], 1)

    # ------------------------------------------------------------------ GST
    def gst(self, style_mel):
        """GST.forward (layers/gst_layers.py:17-21) for one style mel [Ts, 80] -> [256]."""
        w = self.w
        x = np.asarray(style_mel, self.dt)[None]  # [C=1, H=Ts, W=80] (ReferenceEncoder.forward :58-61)
        for i in range(6):
            W, b = w[f"gst.encoder.convs.{i}.weight"], w[f"gst.encoder.convs.{i}.bias"]
            _, Hh, Ww = x.shape
            Ho, Wo = (Hh - 1) // 2 + 1, (Ww - 1) // 2 + 1  # k=3, stride 2, pad 1
            xp = np.pad(x, ((0, 0), (1, 1), (1, 1)))
            y = np.zeros((W.shape[0], Ho, Wo), self.dt)
            for ki in range(3):
                for kj in range(3):
                    patch = xp[:, ki:ki + 2 * (Ho - 1) + 1:2, kj:kj + 2 * (Wo - 1) + 1:2]
                    y += np.einsum("oc,chw->ohw", W[:, :, ki, kj], patch)
            y += b[:, None, None]
            x = np.maximum(self._bn(f"gst.encoder.bns.{i}", y, 1e-5), 0)
        seq = x.transpose(1, 0, 2).reshape(x.shape[1], -1)  # [H6, 128 * W6] (:67-72)
        h = self._gru_seq("gst.encoder.recurrence", seq)[-1]
        # StyleTokenLayer + MultiHeadAttention (:88-168)
        tokens = np.tanh(w["gst.style_token_layer.style_tokens"])
        q = w["gst.style_token_layer.attention.W_query.weight"] @ h
        keys = tokens @ w["gst.style_token_layer.attention.W_key.weight"].T
        vals = tokens @ w["gst.style_token_layer.attention.W_value.weight"].T
        out = np.zeros(256, self.dt)
        for hd in range(4):
            sl = slice(64 * hd, 64 * hd + 64)
            p = _softmax(keys[:, sl] @ q[sl] / 8.0)  # key_dim ** 0.5 = 8
            out[sl] = p @ vals[:, sl]
        return out

    # ------------------------------------------------------------------ encoder
    def encoder(self, ids, speaker_id=None, style_mel=None):
        """embedding -> Encoder -> + speaker embedding -> + GST (models/tacotrongst.py:65-73)."""
        x = self.w["embedding.weight"][np.asarray(ids)]
        x = self._prenet("encoder.prenet", x)
        out = self.cbhg("encoder.cbhg.cbhg", x, 16, [128, 128])
        if speaker_id is not None and "speaker_embedding.weight" in self.w:
            out = out + self.w["speaker_embedding.weight"][speaker_id][None, :]
        if style_mel is not None:
            out = out + self.gst(style_mel)[None, :]
        return out

    # ------------------------------------------------------------------ decoder
    def _attention(self, st, h_att, inputs, P):
        """Attention.forward (layers/common_layers.py:225-256), mask=None at inference."""
        w = self.w
        dt = self.dt
        L = inputs.shape[0]
        pq = w["decoder.attention_layer.query_layer.linear_layer.weight"] @ h_att
        pre = pq[None, :] + P
        if self.location_attn:
            cat = np.stack([st["att_w"], st["att_cum"]])
            cw = w["decoder.attention_layer.location_layer.location_conv.weight"]
            pad = (cw.shape[2] - 1) // 2
            catp = np.pad(cat, ((0, 0), (pad, pad)))
            conv = np.zeros((cw.shape[0], L), dt)
            for j in range(cw.shape[2]):
                conv += cw[:, :, j] @ catp[:, j:j + L]
            loc = conv.T @ w["decoder.attention_layer.location_layer.location_dense.linear_layer.weight"].T
            pre = pq[None, :] + loc + P
        e = np.tanh(pre) @ w["decoder.attention_layer.v.linear_layer.weight"][0] + \
            w["decoder.attention_layer.v.linear_layer.bias"][0]
        if self.attn_win:
            back, front = st["win_idx"] - 2, st["win_idx"] + 6
            if back > 0:
                e[:back] = -np.inf
            if front < L:
                e[front:] = -np.inf
            if st["win_idx"] == -1:
                e[0] = e.max()
            st["win_idx"] = int(np.argmax(e))
        if self.attn_norm == "softmax":
            align = _softmax(e)
        elif self.attn_norm == "sigmoid":
            s = _sig(e)
            align = s / s.sum()
        else:
            raise RuntimeError("Unknown value for attention norm type")
        if self.location_attn:
            st["att_cum"] = st["att_cum"] + align
        if self.forward_attn:
            alpha, u = st["alpha"], st["u"]
            prev = np.concatenate([[0.0], alpha[:-1]]).astype(dt)
            a = ((1 - u) * alpha + u * prev + 1e-8) * align
            if self.forward_attn_mask:
                n = int(np.argmax(prev))
                val = a.max()
                a[n + 3:] = 0
                if n >= 1:
                    a[:n - 1] = 0
                else:
                    a[:L - 1] = 0
                a[(n - 2) % L] = 0.01 * val
            st["alpha"] = a / a.sum()
            ctx = st["alpha"] @ inputs
            if self.trans_agent:
                ta = w["decoder.attention_layer.ta.weight"][0] @ np.concatenate([ctx, h_att]) + \
                    w["decoder.attention_layer.ta.bias"][0]
                st["u"] = _sig(ta)
            st["att_w"] = st["alpha"]
        else:
            ctx = align @ inputs
            st["att_w"] = align
        return ctx

    def decoder(self, memory_in):
        """Decoder.inference (layers/tacotron.py:439-470) for one sentence.
        memory_in [L, 256] -> mel [T*r, 80], stop [T], align [T, L]."""
        w = self.w
        dt = self.dt
        inputs = memory_in.astype(dt)
        L = inputs.shape[0]
        P = inputs @ w["decoder.attention_layer.inputs_layer.linear_layer.weight"].T
        # _init_states (:336-357) + Attention.init_states (common_layers.py:152-161)
        memory = w["decoder.memory_init.weight"][0].copy()
        h_att = w["decoder.attention_rnn_init.weight"][0].copy()
        h_dec = [w["decoder.decoder_rnn_inits.weight"][i].copy() for i in range(2)]
        ctx = np.zeros(inputs.shape[1], dt)
        alpha = np.concatenate([[1.0], np.zeros(L - 1) + 1e-7]).astype(np.float32).astype(dt)
        st = dict(att_w=np.zeros(L, dt), att_cum=np.zeros(L, dt), alpha=alpha, u=0.5, win_idx=-1)
        outs, stops, aligns = [], [], []
        t = 0
        while True:
            x = self._prenet("decoder.prenet", memory)  # decode() (:366-394)
            p = [w[f"decoder.attention_rnn.{n}"] for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
            h_att = self._gru_cell(np.concatenate([x, ctx]), h_att, *p)
            ctx = self._attention(st, h_att, inputs, P)
            d = w["decoder.project_to_decoder_in.weight"] @ np.concatenate([h_att, ctx]) + \
                w["decoder.project_to_decoder_in.bias"]
            for i in range(2):
                p = [w[f"decoder.decoder_rnns.{i}.{n}"] for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
                h_dec[i] = self._gru_cell(d, h_dec[i], *p)
                d = h_dec[i] + d
            out = _sig(w["decoder.proj_to_mel.weight"] @ d + w["decoder.proj_to_mel.bias"])
            stop = _sig(w["decoder.stopnet.linear.weight"][0] @ np.concatenate([d, out]) +
                        w["decoder.stopnet.linear.bias"][0])
            outs.append(out)
            stops.append(stop)
            aligns.append(st["att_w"].copy())
            t += 1
            if t > L / 4 and (stop > 0.6 or st["att_w"][-1] > 0.6):  # (:464-469)
                break
            elif t > self.max_decoder_steps:
                break
            memory = np.concatenate([memory[self.r * 80:], out])  # _update_memory_queue (:396-404)
        mel = np.stack(outs).reshape(-1, 80)
        return mel, np.array(stops), np.stack(aligns)

    # ------------------------------------------------------------------ postnet
    def postnet(self, mel):
        """PostCBHG + last_linear + sigmoid (models/tacotrongst.py:76-78).  [T, 80] -> [T, 1025]."""
        y = self.cbhg("postnet.cbhg", np.asarray(mel, self.dt), 8, [256, 80])
        return _sig(y @ self.w["last_linear.0.weight"].T + self.w["last_linear.0.bias"])

    def inference(self, ids, speaker_id=None, style_mel=None):
        enc = self.encoder(ids, speaker_id, style_mel)
        mel, stop, align = self.decoder(enc)
        return dict(enc=enc, mel=mel, linear=self.postnet(mel), stop=stop, align=align)
