"""Measurement (GPU box): per-fixture parity of every reference-run model fixture on every path
that serves it, as JSON lines — the numbers the test tolerances are set from.

For each tests/golden fixture family:
  t2_*   Decoder.inference + Postnet from the reference's encoder output (resident: the mask form or
         the general form; multi-launch: TTS_RESIDENT=0) and Tacotron2.inference end to end (resident);
  t2bn_* prenet_type "bn": inference end to end (resident) and a batch of two (multi-launch);
  t2spk_* speaker embeddings: inference_batch with the speaker id (resident, multi-launch);
  tf_*   teacher-forced Decoder.forward (multi-launch step kernels);
  trunc_t2_3texts  inference_truncated over three texts (resident);
  gst_* / taco_*  Tacotron / TacotronGST inference end to end (resident GST decoder) and decoder +
         PostCBHG from the reference's encoder output (resident, multi-launch).
Metrics: exact frame / step counts, exact per-step attention argmax, exact stop decisions (0.5 for
Tacotron2, 0.6 for Tacotron), relative RMS of mel / mel_post / linear, max-abs of alignments and
stop probabilities (Tacotron2 teacher forcing: stop logits, max-abs relative to max |logit|).

    python tools/parity_report.py profiles/r05_parity_report.jsonl
"""
import glob
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
from conftest import GOLDEN, golden, golden_flags, load_pkg, rel_rms, weights_mod  # noqa: E402

OUT = []


def emit(**kw):
    for k, v in list(kw.items()):
        if isinstance(v, (np.floating, np.bool_)):
            kw[k] = v.item()
        if isinstance(v, float):
            kw[k] = float(f"{v:.3e}")
    OUT.append(kw)
    print(json.dumps(kw), flush=True)


class env:
    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def names(pat):
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, pat)))


def t2_model(fl, warm=True, num_speakers=0, prenet_type="original", sd=None, max_batch=1):
    t2 = load_pkg("tacotron2")
    m = t2.Tacotron2(130, num_speakers, r=1, attn_win=fl["attn_win"], attn_norm=fl["attn_norm"],
                     forward_attn=fl["forward_attn"], trans_agent=fl["trans_agent"],
                     forward_attn_mask=fl["forward_attn_mask"], location_attn=fl["location_attn"],
                     prenet_type=prenet_type)
    if sd is not None:
        m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.decoder.max_decoder_steps = fl["max_decoder_steps"]
    m.max_len = 256
    m.max_batch = max_batch
    m = m.cuda().eval()
    if warm:
        m.inference_batch([[5, 6]] * max_batch)  # handles created inside the caller's env block
    return m


def t2_metrics(fixture, path, out, b, z, L):
    T = out["frames"][b]
    ok_T = T == z["mel"].shape[0]
    d = dict(fixture=fixture, path=path, frames_exact=bool(ok_T))
    if not ok_T:
        emit(**d)
        return
    al = out["align"][b, :T, :L].cpu().numpy()
    st = out["stop"][b, :T].cpu().numpy()
    emit(**d, argmax_exact=bool(np.array_equal(al.argmax(1), z["align"].argmax(1))),
         stop_exact=bool(np.array_equal(st > 0.5, z["stop"] > 0.5)),
         mel_rel=rel_rms(out["mel"][b, :T].cpu().numpy(), z["mel"]),
         mel_post_rel=rel_rms(out["mel_post"][b, :T].cpu().numpy(), z["mel_post"]),
         align_maxabs=float(np.abs(al - z["align"]).max()), stop_maxabs=float(np.abs(st - z["stop"]).max()))


def general(fl):
    """the resident decoder's general attention form serves it (not synthesize.py's masked one)"""
    return not (fl["forward_attn"] and fl["forward_attn_mask"] and fl["attn_norm"] == "sigmoid"
                and not fl["location_attn"] and not fl["attn_win"] and not fl["trans_agent"])


def tacotron2_cases():
    for c in names("t2_*.npz"):
        z = golden(c)
        fl = golden_flags(z)
        L = len(z["ids"])
        enc = torch.from_numpy(z["enc"]).cuda()[None]
        for path, e in (("resident", {}), ("multi_launch", {"TTS_RESIDENT": "0"})):
            with env(**e):
                m = t2_model(fl)
            out = m.inference_batch(None, enc=enc, lens=[L])
            assert bool(m.last_timing["resident"]) == (path == "resident"), (c, path)
            t2_metrics(c, path + ("_general" if path == "resident" and general(fl) else ""), out, 0, z, L)
            if path == "resident":
                mel, mel_post, align, stop = m.inference(torch.from_numpy(z["ids"])[None])
                o = dict(frames=[mel.shape[1]], mel=mel, mel_post=mel_post, align=align, stop=stop[..., 0])
                t2_metrics(c, "resident_end_to_end", o, 0, z, L)
            del m


def bn_cases():
    sd = weights_mod().tacotron2_weights(0, prenet_bn=True)
    for c in names("t2bn_*.npz"):
        z = golden(c)
        fl = golden_flags(z)
        m = t2_model(fl, prenet_type="bn", sd=sd)
        mel, mel_post, align, stop = m.inference(torch.from_numpy(z["ids"])[None])
        t2_metrics(c, "resident_end_to_end", dict(frames=[mel.shape[1]], mel=mel, mel_post=mel_post, align=align,
                                                  stop=stop[..., 0]), 0, z, len(z["ids"]))
        m = t2_model(fl, prenet_type="bn", sd=sd, max_batch=2)
        out = m.inference_batch([z["ids"], z["ids"]])
        t2_metrics(c, "multi_launch_batch2", out, 1, z, len(z["ids"]))


def speaker_cases():
    sd = weights_mod().tacotron2_weights(0, num_speakers=4)
    for c in names("t2spk_*.npz"):
        z = golden(c)
        fl = golden_flags(z)
        for path, e in (("resident", {}), ("multi_launch", {"TTS_RESIDENT": "0"})):
            with env(**e):
                m = t2_model(fl, num_speakers=4, sd=sd)
            out = m.inference_batch([z["ids"]], speaker_ids=[int(z["speaker_id"])])
            t2_metrics(c, path + "_end_to_end", out, 0, z, len(z["ids"]))


def teacher_cases():
    for c in names("tf_*.npz"):
        z = golden(c)
        m = t2_model(golden_flags(z))
        mel, stop, align = m.decoder_forward(torch.from_numpy(z["enc"])[None], torch.from_numpy(z["teacher"])[None])
        al = align[0].cpu().numpy()
        emit(fixture=c, path="teacher_forcing", argmax_exact=bool(np.array_equal(al.argmax(1), z["align"].argmax(1))),
             mel_rel=rel_rms(mel[0].cpu().numpy(), z["mel"]), align_maxabs=float(np.abs(al - z["align"]).max()),
             stop_logit_rel_maxabs=float(np.abs(stop[0].cpu().numpy() - z["stop"]).max() / max(1.0, np.abs(z["stop"]).max())))


def truncated_case():
    z = golden("trunc_t2_3texts")
    m = t2_model(golden_flags(z))
    for i in range(3):
        mel, mel_post, align, stop = m.inference_truncated(torch.from_numpy(z[f"ids{i}"])[None])
        ok = mel.shape[1] == z[f"mel{i}"].shape[0]
        d = dict(fixture=f"trunc_t2_3texts[{i}]", path="resident_truncated", frames_exact=bool(ok))
        if ok:
            d.update(argmax_exact=bool(np.array_equal(align[0].cpu().numpy().argmax(1), z[f"align{i}"].argmax(1))),
                     mel_rel=rel_rms(mel[0].cpu().numpy(), z[f"mel{i}"]),
                     mel_post_rel=rel_rms(mel_post[0].cpu().numpy(), z[f"mel_post{i}"]))
        emit(**d)


def tacotron_cases():
    t = load_pkg("tacotron")
    for c in names("gst_*.npz") + names("taco_*.npz"):
        z = golden(c)
        fl = golden_flags(z)
        L = len(z["ids"])
        sid = int(z["speaker_id"])
        sid = None if sid < 0 else torch.tensor([sid])
        style = torch.from_numpy(z["style_mel"])[None] if "style_mel" in z else None

        def build():
            cls = t.TacotronGST if fl["model"] == "TacotronGST" else t.Tacotron
            m = cls(130, fl["num_speakers"], r=fl["r"], memory_size=fl["memory_size"], attn_win=fl["attn_win"],
                    attn_norm=fl["attn_norm"], forward_attn=fl["forward_attn"], trans_agent=fl["trans_agent"],
                    forward_attn_mask=fl["forward_attn_mask"], location_attn=fl["location_attn"],
                    prenet_type=fl.get("prenet_type", "original"))
            m.decoder.max_decoder_steps = fl["max_decoder_steps"]
            return m.cuda().eval()

        def metrics(path, mel, lin, align, stop):
            d = dict(fixture=c, path=path, steps_exact=bool(align.shape[0] == z["align"].shape[0]))
            if d["steps_exact"]:
                d.update(argmax_exact=bool(np.array_equal(align[:, :L].argmax(1), z["align"].argmax(1))),
                         stop_exact=bool(np.array_equal(stop > 0.6, z["stop"] > 0.6)),
                         mel_rel=rel_rms(mel, z["mel"]), align_maxabs=float(np.abs(align[:, :L] - z["align"]).max()),
                         stop_maxabs=float(np.abs(stop - z["stop"]).max()))
                if lin is not None:
                    d["linear_rel"] = rel_rms(lin, z["linear"])
            emit(**d)

        m = build()
        x = torch.from_numpy(z["ids"])[None]
        if fl["model"] == "TacotronGST":
            mel, lin, align, stop = m.inference(x, speaker_ids=sid, style_mel=style)
        else:
            mel, lin, align, stop = m.inference(x, speaker_ids=sid)
        metrics("resident_end_to_end", mel[0].cpu().numpy(), lin[0].cpu().numpy(), align[0].cpu().numpy(),
                stop[0].cpu().numpy())
        for path, e in (("resident", {}), ("multi_launch", {"TTS_RESIDENT": "0"})):
            with env(**e):
                m = build()
                out = m.inference_batch(None, enc=torch.from_numpy(z["enc"])[None].cuda(), lens=[L], postnet=False)
            melz = torch.from_numpy(z["mel"])[None].cuda()
            lin = m.postnet(melz, [melz.shape[1]])
            metrics(path, out["mel"][0].cpu().numpy(), lin[0].cpu().numpy(), out["align"][0].cpu().numpy(),
                    out["stop"][0].cpu().numpy())


if __name__ == "__main__":
    for fn in (tacotron2_cases, bn_cases, speaker_cases, teacher_cases, truncated_case, tacotron_cases):
        fn()
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            for r in OUT:
                f.write(json.dumps(r) + "\n")
    worst = {}
    for r in OUT:
        for k, v in r.items():
            if isinstance(v, float):
                worst[k] = max(worst.get(k, 0.0), v)
    bad = [r for r in OUT if any(v is False for v in r.values())]
    print(json.dumps({"rows": len(OUT), "worst": worst, "inexact_rows": bad}))
