"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference synthesis path.

This package is the parity *checker* for the MI355X path.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it, and only
to check or to time the CPU baseline.  The product package (``your-voice-tts_amd``) never
imports, links or executes anything under ``oracle/``: it fails loudly when its HIP library
is missing instead of falling back to the CPU.

* ``tacotron2_oracle`` — numpy restatement of ``Tacotron2.inference``
  (``models/tacotron2.py:62-73``): encoder, autoregressive ``Decoder.inference`` with every
  ``Attention`` variant, Postnet.  Pinned against ``tests/golden/t2_*.npz``, which
  ``tests/golden/make_golden.py`` produced by running the reference itself (imported here
  with the text front-end stubbed) on weights from ``weights.py``'s deterministic generator.
* ``griffin_lim_oracle`` — numpy/scipy restatement of ``AudioProcessor.inv_mel_spectrogram``
  / ``inv_spectrogram`` (``utils/audio.py:96-201``) and of the librosa 0.6.2 functions they
  call (``filters.mel``, ``stft``, ``istft``, ``window_sumsquare``).  librosa is absent from
  this image, so the librosa half is *parity unpinned*; the reference's own glue
  (denormalise, dB->amp, pinv, power, GL loop, ``lfilter`` inverse pre-emphasis) is pinned by
  ``tests/golden/gl_*.npz`` (reference ``utils/audio.py`` executed with this restatement
  standing in for librosa).
"""
