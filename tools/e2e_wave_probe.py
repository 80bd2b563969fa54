"""Measurement (GPU box): end-to-end waveform distance to the oracle chain over several numpy phase
draws, and the mel_post distance, for the t2_fwdmask fixtures (python tools/e2e_wave_probe.py)."""
import os, sys
import numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from conftest import golden, golden_flags, load_pkg, rel_rms, tacotron2_config
from oracle.griffin_lim_oracle import AudioOracle
cfg = tacotron2_config()["audio"]
t2 = load_pkg("tacotron2")
for case in ("t2_fwdmask_L12", "t2_fwdmask_L40", "t2_fwdmask_L100"):
    z = golden(case); fl = golden_flags(z)
    m = t2.Tacotron2(130, 0, r=1, attn_win=fl["attn_win"], attn_norm=fl["attn_norm"], forward_attn=fl["forward_attn"],
                     trans_agent=fl["trans_agent"], forward_attn_mask=fl["forward_attn_mask"], location_attn=fl["location_attn"])
    m.decoder.max_decoder_steps = fl["max_decoder_steps"]; m = m.cuda().eval()
    ap = load_pkg("audio").AudioProcessor(**cfg)
    errs = []
    for seed in (3, 4, 5, 6):
        np.random.seed(seed)
        wavs, info = load_pkg("synthesis").synthesize_batch(m, ap, [z["ids"]], phase="numpy")
        np.random.seed(seed)
        ref = AudioOracle(**cfg).inv_mel_spectrogram(z["mel_post"].T)
        errs.append(rel_rms(wavs[0], ref))
    out = m.inference_batch([z["ids"]])
    mp = out["mel_post"][0, :z["mel"].shape[0]].cpu().numpy()
    print(case, os.environ.get("TTS_PROJ_VALU", "0"), "mel_post", rel_rms(mp, z["mel_post"]), "wav", ["%.2e" % e for e in errs], flush=True)
