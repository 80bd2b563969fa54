import sys, os
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import numpy as np, torch, pathlib, tempfile
from conftest import load_pkg
from test_cli import _write_model_files
synth = load_pkg("synthesis"); gu = load_pkg("generic_utils")
tmp = pathlib.Path(tempfile.mkdtemp())
cfg_path, ckpt, _ = _write_model_files(tmp)
conf = tmp / "conf.json"
conf.write_text('{"tts_path": "%s", "tts_file": "%s", "tts_config": "config.json", "wavernn_lib_path": "", "use_cuda": true, "port": 5002}' % (tmp, ckpt.name))
s = synth.Synthesizer(gu.load_config(str(conf)))
m = s.tts_model
print("flags", m.flags)
sens = s.sentences("It took me quite a long time to develop a voice and now that I have it I am not silent.")
ids = [np.asarray(s.input_adapter(x)) for x in sens]
print("lens", [len(i) for i in ids])
out = m.inference_batch(ids)
print("frames", out["frames"], m.last_timing)
out = m.inference_batch(ids)
print("frames", out["frames"], m.last_timing)
