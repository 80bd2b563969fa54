// fp32 MFMA implicit-GEMM Conv1d over time-major activations [B][T][C] ("same" padding per
// sentence length: rows t >= T_b read as zero), with a folded-BatchNorm epilogue.
// Used by the Postnet (layers/tacotron2.py:30-45), the encoder convolutions (:48-76) and, with
// KW = 1, the encoder LSTM input projection.
#pragma once
#include "common.h"

namespace tts {

enum ConvAct { CONV_NONE = 0, CONV_RELU = 1, CONV_TANH = 2 };

struct ConvArgs {
    const float* in;     // [B][Tmax][Cin] (ignored when ids is set)
    const int* ids;      // optional [B][Tmax] row ids into `table` (fused embedding gather)
    const float* table;  // [rows][Cin]
    float* out;          // [B][Tmax][Cout]
    const float* W;      // packed [Cin][KW][co_pad]
    const float* scale;  // [Cout] (null = 1)
    const float* shift;  // [Cout] (null = 0)
    const float* resid;  // [B][Tmax][Cout] or null: out = resid + y
    const int* T;        // [B] valid frames per sentence
    int Tmax, Cin, Cout, co_pad, act;
};

constexpr int CONV_BN = 64;  // output channels per tile
inline int conv_co_pad(int Cout) { return (Cout + CONV_BN - 1) / CONV_BN * CONV_BN; }

// W [Cout][Cin][KW] (PyTorch Conv1d layout) -> packed [Cin][KW][co_pad]
hipError_t conv_pack(const float* W, int Cout, int Cin, int KW, float* out, hipStream_t s);
// W [Cout][Cin] (Linear layout, rows stacked into Cout) -> packed [Cin][1][co_pad]
hipError_t linear_pack_as_conv(const float* W, int Cout, int Cin, int co_offset, int co_pad, float* out,
                               hipStream_t s);
// scale = gamma / sqrt(var + eps); shift = beta + (bias - mean) * scale
hipError_t fold_bn(const float* bias, const float* gamma, const float* beta, const float* mean, const float* var,
                   int C, float* scale, float* shift, hipStream_t s);
// KW in {1, 5}.  frames_hint = sum of T_b picks the tile height (small batches: 16 frames).
hipError_t conv_launch(const ConvArgs& a, int KW, int B, int frames_hint, hipStream_t s);

}  // namespace tts
