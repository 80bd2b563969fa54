import os, sys, json
sys.path.insert(0, "tests")
import torch
from conftest import load_pkg, golden, golden_flags
t2 = load_pkg("tacotron2")
fl = golden_flags(golden("t2_fwdmask_L100"))
m = t2.Tacotron2(130, 0, r=1, attn_win=fl["attn_win"], attn_norm=fl["attn_norm"], forward_attn=fl["forward_attn"],
                 trans_agent=fl["trans_agent"], forward_attn_mask=fl["forward_attn_mask"], location_attn=fl["location_attn"])
m.decoder.max_decoder_steps = 1000
m.cuda().eval()
ids = torch.from_numpy(golden("t2_fwdmask_L100")["ids"])[None]
for _ in range(3):
    m.inference(ids)
p = m.profile_resident_phases()
for k in ("cu0", "attention_cu"):
    print(k, {a: round(b, 3) for a, b in p[k].items()})
