"""Config surface of the reference (utils/generic_utils.py:18-32, 254-289), unchanged formats.

``load_config`` accepts the reference's JSON files as they are (``//`` comments and backslash
line continuations stripped, as utils/generic_utils.py:24-32).  ``setup_model`` accepts both the
3-argument signature of the reference function (``setup_model(num_chars, num_speakers, c)``)
and the 2-argument call its callers make (``synthesize.py:93``, ``server/synthesizer.py:55``),
which raises TypeError in the reference; ``c.num_speakers`` may be absent (it is absent from
every reference config, generic_utils.py:278).
"""
from __future__ import annotations

import json
import os
import re

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CONFIG_DIR = os.path.join(PKG_DIR, "configs")


class AttrDict(dict):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.__dict__ = self


def load_config(config_path: str) -> AttrDict:
    with open(config_path, "r") as f:
        s = f.read()
    s = re.sub(r"\\\n", "", s)
    s = re.sub(r"//.*\n", "\n", s)
    cfg = AttrDict()
    cfg.update(json.loads(s))
    return cfg


def default_config(name: str = "config_tacotron2.json") -> AttrDict:
    return load_config(os.path.join(CONFIG_DIR, name))


def setup_model(num_chars, num_speakers_or_c, c=None, **kw):
    if c is None:
        c, num_speakers = num_speakers_or_c, getattr(num_speakers_or_c, "num_speakers", 0) or 0
    else:
        num_speakers = num_speakers_or_c
    model = c.model.lower()
    if model == "tacotron2":
        from .tacotron2 import Tacotron2
        return Tacotron2(num_chars=num_chars, num_speakers=num_speakers, r=c.r, attn_win=c.windowing,
                         attn_norm=c.attention_norm, prenet_type=c.prenet_type, prenet_dropout=c.prenet_dropout,
                         forward_attn=c.use_forward_attn, trans_agent=c.transition_agent,
                         forward_attn_mask=c.forward_attn_mask, location_attn=c.location_attn,
                         separate_stopnet=c.separate_stopnet, **kw)
    if model in ("tacotron", "tacotrongst"):  # utils/generic_utils.py:258-274
        from .tacotron import Tacotron, TacotronGST
        cls = TacotronGST if model == "tacotrongst" else Tacotron
        return cls(num_chars=num_chars, num_speakers=num_speakers, r=c.r, linear_dim=1025, mel_dim=80,
                   memory_size=c.memory_size, attn_win=c.windowing, attn_norm=c.attention_norm,
                   prenet_type=c.prenet_type, prenet_dropout=c.prenet_dropout, forward_attn=c.use_forward_attn,
                   trans_agent=c.transition_agent, forward_attn_mask=c.forward_attn_mask,
                   location_attn=c.location_attn, separate_stopnet=c.separate_stopnet, **kw)
    raise NotImplementedError(f"model {c.model!r} is not one of Tacotron2, Tacotron, TacotronGST")
