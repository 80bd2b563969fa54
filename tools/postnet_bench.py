"""Postnet / encoder launch timing at batch 1 (measurement only, GPU box): mean ms per call of
tts_postnet_run on a T-frame mel and of Tacotron2.encode on an L-id sentence, over many calls
back to back (HIP events on the caller's stream).  python tools/postnet_bench.py [T] [L]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import load_pkg, weights_mod  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 222
L = int(sys.argv[2]) if len(sys.argv) > 2 else 100
gu = load_pkg("generic_utils")
_native = load_pkg("_native")
cfg = gu.default_config("config_tacotron2.json")
cfg.forward_attn_mask = True
m = gu.setup_model(130, cfg, max_batch=1, max_len=256).cuda().eval()
lib, hdec, hpost = m._handles(L, 1)
mel = torch.randn(1, T, 80, device="cuda")
out = torch.empty_like(mel)
Tarr = _native.i32_array([T])


def post():
    _native.check(lib.tts_postnet_run(hpost, ctypes.c_void_p(mel.data_ptr()), Tarr, 1, T, ctypes.c_void_p(out.data_ptr()),
                                      _native.stream_handle()), "postnet")


ids = torch.from_numpy(weights_mod().synthetic_ids(L, 1)[None]).cuda()


def enc():
    m.encode(ids, [L])


res = {}
for name, fn in (("postnet", post), ("encoder", enc)):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 200
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    res[name] = round(e0.elapsed_time(e1) / n * 1e3, 1)
print("us per call", res, "T", T, "L", L, {k: os.environ.get(k) for k in ("TTS_CONV_SMALL", "TTS_CONV_FUSED_REDUCE", "TTS_CONV_NSMAX")})
