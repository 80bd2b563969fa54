"""MI355X-native Tacotron2 + Griffin-Lim synthesis path (drop-in for prototypefund/your-voice-TTS).

The compute runs in ``libtts_hip.so`` (hand-written HIP for gfx950, C-ABI declared in
``include/tts_hip.h``); this package is the host side that mirrors the reference's Python
interface for the path:

* ``tacotron2.Tacotron2``           <- ``models/tacotron2.py`` (``inference``, state_dict keys)
* ``audio.AudioProcessor``          <- ``utils/audio.py`` (``inv_mel_spectrogram``, ``inv_spectrogram``)
* ``synthesis.synthesis / tts``     <- ``utils/synthesis.py``, ``synthesize.py``
* ``synthesis.Synthesizer``         <- ``server/synthesizer.py``
* ``generic_utils.load_config / setup_model`` <- ``utils/generic_utils.py``

The directory name is not a Python identifier; import with
``importlib.import_module("your-voice-tts_amd")``.  Importing is cheap; the native library is
loaded on first use and a missing or unloadable library raises (there is no CPU fallback).
"""
import sys as _sys

_sys.modules.setdefault("yvtts_amd", _sys.modules[__name__])

__all__ = ["weights", "generic_utils", "tacotron2", "audio", "synthesis", "sharding"]
