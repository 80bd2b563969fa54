#!/usr/bin/env python3
"""Print the measured parity errors of the HIP path (GPU box): per golden case the frame count,
argmax-path equality and the float errors that tests/test_gpu_parity.py bounds, plus the
end-to-end waveform error.  Output is JSON lines (copied into DESIGN.md / profiles/)."""
import glob
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import golden, golden_flags, load_pkg, rel_rms, tacotron2_config  # noqa: E402
from oracle.griffin_lim_oracle import AudioOracle  # noqa: E402


def main():
    t2 = load_pkg("tacotron2")
    audio = load_pkg("audio")
    cfg = tacotron2_config()["audio"]
    for path in sorted(glob.glob(os.path.join(REPO, "tests", "golden", "t2_*.npz"))):
        name = os.path.basename(path)[:-4]
        z = golden(name)
        fl = golden_flags(z)
        m = t2.Tacotron2(130, 0, r=1, attn_win=fl["attn_win"], attn_norm=fl["attn_norm"],
                         forward_attn=fl["forward_attn"], trans_agent=fl["trans_agent"],
                         forward_attn_mask=fl["forward_attn_mask"], location_attn=fl["location_attn"]).cuda()
        m.decoder.max_decoder_steps = fl["max_decoder_steps"]
        out = m.inference_batch(None, enc=torch.from_numpy(z["enc"]).cuda()[None], lens=[len(z["ids"])])
        T = out["frames"][0]
        L = len(z["ids"])
        al = out["align"][0, :T, :L].cpu().numpy()
        rec = dict(case=name, frames=T, ref_frames=int(z["mel"].shape[0]),
                   argmax_path_equal=bool((al.argmax(1) == z["align"].argmax(1)).all()),
                   stop_decisions_equal=bool(((out["stop"][0, :T].cpu().numpy() > 0.5) == (z["stop"] > 0.5)).all()),
                   mel_rel_rms=rel_rms(out["mel"][0, :T].cpu().numpy(), z["mel"]),
                   mel_post_rel_rms=rel_rms(out["mel_post"][0, :T].cpu().numpy(), z["mel_post"]),
                   align_max_abs=float(np.abs(al - z["align"]).max()),
                   stop_max_abs=float(np.abs(out["stop"][0, :T].cpu().numpy() - z["stop"]).max()))
        print(json.dumps(rec))
    for path in sorted(glob.glob(os.path.join(REPO, "tests", "golden", "gl_*mel*.npz"))):
        name = os.path.basename(path)[:-4]
        z = golden(name)
        ap = audio.AudioProcessor(**{**cfg, "griffin_lim_iters": int(z["iters"])})
        np.random.seed(int(z["phase_seed"]))
        wav = ap.inv_mel_spectrogram(z["mel"])
        print(json.dumps(dict(case=name, wav_rel_rms=rel_rms(wav, z["wav"]))))
    # end to end (ids -> wav), 60 GL iterations, vs the oracle chain on the reference's mel_post
    z = golden("t2_fwdmask_L12")
    fl = golden_flags(z)
    m = t2.Tacotron2(130, 0, r=1, attn_norm=fl["attn_norm"], forward_attn=True, forward_attn_mask=True,
                     location_attn=False).cuda()
    ap = audio.AudioProcessor(**cfg)
    np.random.seed(3)
    wavs, info = load_pkg("synthesis").synthesize_batch(m, ap, [z["ids"]], phase="numpy")
    np.random.seed(3)
    ref = AudioOracle(**cfg).inv_mel_spectrogram(z["mel_post"].T)
    print(json.dumps(dict(case="end_to_end_L12_gl60", wav_rel_rms=rel_rms(wavs[0], ref))))
    # run-to-run determinism: decoder from fixed encoder outputs, encoder, whole chain
    enc = torch.from_numpy(z["enc"]).cuda()[None]
    a1 = m.inference_batch(None, enc=enc, lens=[len(z["ids"])])["mel_post"].cpu().numpy()
    a2 = m.inference_batch(None, enc=enc, lens=[len(z["ids"])])["mel_post"].cpu().numpy()
    ids = torch.from_numpy(z["ids"]).cuda()[None]
    e1 = m.encode(ids, [len(z["ids"])]).cpu().numpy()
    e2 = m.encode(ids, [len(z["ids"])]).cpu().numpy()
    np.random.seed(3)
    w2, _ = load_pkg("synthesis").synthesize_batch(m, ap, [z["ids"]], phase="numpy")
    print(json.dumps(dict(case="determinism", decoder_postnet_bitwise=bool((a1 == a2).all()),
                          encoder_bitwise=bool((e1 == e2).all()), encoder_max_abs=float(np.abs(e1 - e2).max()),
                          end_to_end_bitwise=bool((wavs[0] == w2[0]).all()),
                          end_to_end_rerun_rel=rel_rms(w2[0], ref))))


if __name__ == "__main__":
    main()
