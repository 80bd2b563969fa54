#!/usr/bin/env python3
"""Per-kernel HBM bytes per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_summary.py FETCH_counter_collection.csv WRITE_counter_collection.csv out.json [prefix]

(prefix, e.g. "gst_", is prepended to every label: the names bench.py's load_traffic looks up).
"gl_iter" is one GL iteration as bench.py prices it: the per-frame STFT/iSTFT launch plus the
overlap-add launch (gl_iter_frames + gl_ola).

gfx950 corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE and
WRITE_SIZE are in KiB; FETCH_SIZE reports half the bytes of a wide coalesced read, so
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  Infinity-Cache hits are counted as fabric
traffic (not excluded).  Kernels are labelled with the names bench.py uses.
"""
import csv
import json
import re
import sys
from collections import defaultdict

LABELS = [
    (r"sgemm_kernel<\d+, 0, 0>|sgemm_frag16_kernel<0, 0>", "prenet2"),
    (r"sgemm(?:_frag)?_kernel<\d+, 1, 1>", "att_lstm"),
    (r"sgemm_kernel<\d+, 0, 2>", "query"),
    (r"query_energy_kernel", "query"),
    (r"attention_kernel|attention_fm_kernel", "attention"),
    (r"sgemm(?:_frag)?_kernel<\d+, 1, 3>", "dec_lstm"),
    (r"sgemm_kernel<\d+, 2, 5>|sgemm_frag16_kernel<2, 5>", "mel_fused"),
    (r"sgemm_kernel<\d+, 3, 6>", "enc_lstm"),
    (r"gl_iter_kernel<false|gl_iter_wave_kernel", "gl_iter_frames"),
    (r"gl_iter_kernel<true", "gl_iter_init"),
    (r"gl_persistent_kernel", "gl_persistent"),
    (r"encoder_resident_kernel", "enc_lstm_resident"),
    (r"sgemm_kernel<\d+, 0, 7>", "prenet1"),
    (r"sgemm_kernel<\d+, 0, 8>", "prenet2"),
    (r"sgemm_kernel<\d+, 4, 9>", "att_gru"),
    (r"sgemm_kernel<\d+, 0, 10>", "query"),
    (r"sgemm_kernel<\d+, 0, 11>", "proj"),
    (r"sgemm_kernel<\d+, 4, 12>", "dec_gru"),
    (r"sgemm_kernel<\d+, 0, 13>", "mel"),
    (r"sgemm_kernel<\d+, 2, 14>", "pre1_stop"),
    (r"conv_kernel<5", "conv5"),
    (r"conv_kernel<1", "conv1"),
    (r"gl_magnitude_kernel", "gl_magnitude"),
    (r"preemph_scan_kernel", "preemph"),
    (r"gl_ola_kernel|gl_ola_multi_kernel", "gl_ola"),
    (r"project_inputs_kernel", "project_inputs"),
    (r"resident_decoder_kernel<(?:false|true), true>", "resident_decoder_general"),
    (r"resident_decoder_kernel", "resident_decoder"),
    (r"gl_linear_magnitude_kernel", "gl_linear_magnitude"),
    (r"gl_persistent2_kernel", "gl_persistent2"),
    (r"encoder_resident_batch_kernel", "enc_lstm_resident_batch"),
]


def label(name):
    for pat, lab in LABELS:
        if re.search(pat, name):
            return lab
    return None


def per_kernel(path, counter):
    """mean over dispatches of the counter's per-dispatch sum (summed over its dimensions)."""
    per_dispatch = defaultdict(float)
    names = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            per_dispatch[key] += float(row["Counter_Value"])
            names[key] = row["Kernel_Name"]
    acc = defaultdict(list)
    for k, v in per_dispatch.items():
        lab = label(names[k])
        if lab:
            acc[lab].append(v)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    prefix = sys.argv[4] if len(sys.argv) > 4 else ""
    for d in (fetch, write):
        if "gl_iter_frames" in d and "gl_ola" in d:
            d["gl_iter"] = (d["gl_iter_frames"][0] + d["gl_ola"][0], d["gl_iter_frames"][1])
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes",
           "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 bytes per launch (gfx950 FETCH_SIZE half-count)",
           "per_launch_hbm_bytes": {}, "fetch_kib": {}, "write_kib": {}, "dispatches": {}}
    for k in sorted(set(fetch) | set(write)):
        f, nf = fetch.get(k, (0.0, 0))
        w, nw = write.get(k, (0.0, 0))
        out["per_launch_hbm_bytes"][prefix + k] = (2 * f + w) * 1024
        out["fetch_kib"][prefix + k] = f
        out["write_kib"][prefix + k] = w
        out["dispatches"][prefix + k] = [nf, nw]
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    for k, v in out["per_launch_hbm_bytes"].items():
        print(f"{k:20s} {v / 1e6:10.3f} MB/launch  (fetch {out['fetch_kib'][k]:.0f} KiB, write {out['write_kib'][k]:.0f} KiB)")


if __name__ == "__main__":
    main()
