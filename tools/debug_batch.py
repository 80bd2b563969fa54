"""Debug helper (GPU): per-sentence decoder output in a batch vs the same sentence at batch 1 and
vs the oracle (argmax path, first differing step, mel error)."""
import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
w = importlib.import_module("your-voice-tts_amd.weights")
t2 = importlib.import_module("your-voice-tts_amd.tacotron2")
from oracle.tacotron2_oracle import Tacotron2Oracle  # noqa: E402

fl = dict(attn_norm="sigmoid", forward_attn=True, trans_agent=False, forward_attn_mask=True, location_attn=False)
m = t2.Tacotron2(130, 0, r=1, **fl)
m.load_state_dict({k: torch.from_numpy(v) for k, v in w.tacotron2_weights(0).items()})
m.cuda().eval()
o = Tacotron2Oracle(w.tacotron2_weights(0), dtype=np.float32, attn_win=False, **fl)
lens = w.synthetic_lengths(64, 2)
ids = [w.synthetic_ids(int(L), 100 + b) for b, L in enumerate(lens)]
outB = m.inference_batch(ids)
sel = [int(x) for x in sys.argv[1:]] or [37]
for b in sel:
    L = len(ids[b])
    one = m.inference_batch([ids[b]])
    ref = o.inference(ids[b])
    for name, out, k in (("B=64", outB, b), ("B=1", one, 0)):
        T = out["frames"][k]
        am = out["align"][k, :T, :L].cpu().numpy().argmax(1)
        ra = ref["align"].argmax(1)
        n = min(T, len(ra))
        diff = np.nonzero(am[:n] != ra[:n])[0]
        mel = out["mel"][k, :n].cpu().numpy()
        rel = float(np.sqrt(((mel - ref["mel"][:n]) ** 2).mean() / (ref["mel"][:n] ** 2).mean()))
        step_err = np.abs(mel - ref["mel"][:n]).max(1)
        first_big = int(np.argmax(step_err > 1e-4)) if (step_err > 1e-4).any() else -1
        print(f"sent {b} L={L} {name}: frames {T} ref {ref['mel'].shape[0]} argmax diffs at {diff[:10].tolist()} "
              f"mel rel {rel:.3e} first step err>1e-4: {first_big}", flush=True)
        if len(diff):
            s = diff[0]
            print("   ours  alpha around:", np.round(out["align"][k, s, :L].cpu().numpy()[max(0, am[s] - 3):am[s] + 4], 7))
            print("   oracle alpha around:", np.round(ref["align"][s][max(0, ra[s] - 3):ra[s] + 4], 7))
