"""The ``synthesize.py`` command line (reference synthesize.py:41-146) on the MI355X path.

    python -m your-voice-tts_amd.synthesize "text" config.json checkpoint.pth.tar out_dir/

Same positional arguments and options as the reference: it loads the config and sets
``C.forward_attn_mask = True`` (:85-86), builds the AudioProcessor (:89), sizes the embedding from
the symbol or phoneme table (:92), builds the model with ``setup_model`` and loads ``cp['model']``
(:93-96), runs ``tts`` (Griffin-Lim vocoder, :128-139) and writes
``<text with spaces as underscores, punctuation except '_' removed>.wav`` into ``out_path``
(:141-146).

Differences, each one forced by this tier's scope:
  * the checkpoint is read with ``torch.load(..., weights_only=True)`` (no pickled code runs);
  * the synthesis always runs on the GPU (there is no CPU path), whatever ``--use_cuda`` says;
  * ``--vocoder_path`` (WaveRNN, an external repo that is not part of the reference tree) raises.
"""
from __future__ import annotations

import argparse
import os
import string

import torch

from . import text as _text
from .audio import AudioProcessor
from .generic_utils import load_config, setup_model
from .synthesis import tts


def build_parser():
    """synthesize.py:43-79 (``type=bool`` kept: argparse turns any non-empty string into True)."""
    parser = argparse.ArgumentParser()
    parser.add_argument("text", type=str, help="Text to generate speech.")
    parser.add_argument("config_path", type=str, help="Path to model config file.")
    parser.add_argument("model_path", type=str, help="Path to model file.")
    parser.add_argument("out_path", type=str, help="Path to save final wav file.")
    parser.add_argument("--use_cuda", type=bool, help="Run model on CUDA.", default=False)
    parser.add_argument("--vocoder_path", type=str, default="",
                        help="Path to vocoder model file. If it is not defined, model uses GL as vocoder.")
    parser.add_argument("--vocoder_config_path", type=str, help="Path to vocoder model config file.", default="")
    parser.add_argument("--batched_vocoder", type=bool, default=True,
                        help="If True, vocoder model uses faster batch processing.")
    return parser


def output_file(text: str, out_path: str) -> str:
    """synthesize.py:142-144: spaces -> '_', then every punctuation character except '_' dropped."""
    file_name = text.replace(" ", "_")
    file_name = file_name.translate(str.maketrans("", "", string.punctuation.replace("_", ""))) + ".wav"
    return os.path.join(out_path, file_name)


def load_checkpoint(path: str):
    """``torch.load`` of a reference checkpoint (a dict holding 'model': state_dict) without
    unpickling code; tensors land on the CPU and are moved by ``load_state_dict``."""
    return torch.load(path, map_location="cpu", weights_only=True)


def load_model(C, model_path: str):
    """synthesize.py:92-98 / server/synthesizer.py:49-65: embedding size from the symbol or phoneme
    table, setup_model, cp['model'] into it, eval, on the GPU."""
    model = setup_model(_text.num_chars(C), C)
    cp = load_checkpoint(model_path)
    model.load_state_dict(cp["model"])
    model.eval()
    return model.cuda()


def main(argv=None) -> str:
    args = build_parser().parse_args(argv)
    if args.vocoder_path != "":
        assert args.use_cuda, " [!] Enable cuda for vocoder."
        raise NotImplementedError("WaveRNN vocoder is not part of the reference tree (synthesize.py:12)")
    C = load_config(args.config_path)
    C.forward_attn_mask = True  # synthesize.py:86
    ap = AudioProcessor(**C.audio)
    model = load_model(C, args.model_path)
    print(" > Text: {}".format(args.text))
    _, _, _, wav = tts(model, None, C, None, args.text, ap, args.use_cuda, args.batched_vocoder, figures=False)
    out_path = output_file(args.text, args.out_path)
    print(" > Saving output to {}".format(out_path))
    ap.save_wav(wav, out_path)
    return out_path


if __name__ == "__main__":
    main()
