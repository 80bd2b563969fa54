// fp32 MFMA implicit-GEMM Conv1d over time-major activations [B][T][C] ("same" padding per
// sentence length: rows t >= T_b read as zero), with a folded-BatchNorm epilogue.
// Used by the Tacotron2 Postnet (layers/tacotron2.py:30-45), encoder convolutions (:48-76) and,
// with KW = 1, the encoder LSTM input projection; and by the Tacotron/TacotronGST CBHG stacks
// (layers/tacotron.py:92-206): the conv bank as ONE conv of K taps (bank member k's weights
// centred in the K-tap window, zeros elsewhere), the projections (KW = 3, max-pool fused into the
// input staging), the Highway layers and every Linear (KW = 1).
#pragma once
#include "common.h"

namespace tts {

// CONV_HIGHWAY: GEMM columns interleave a Highway layer's rows (2c = H_c, 2c+1 = T_c) and the
// epilogue writes out[t][c] = relu(H) * sigmoid(T) + resid[t][c] * (1 - sigmoid(T))
// (layers/tacotron.py:86-89) into Cout/2 channels.
enum ConvAct { CONV_NONE = 0, CONV_RELU = 1, CONV_TANH = 2, CONV_SIGMOID = 3, CONV_HIGHWAY = 4 };

struct ConvArgs {
    const float* in;     // [B][Tmax][Cin] (ignored when ids is set)
    const int* ids;      // optional [B][Tmax] row ids into `table` (fused embedding gather)
    const float* table;  // [rows][Cin]
    float* out;          // [B][Tmax][Cout]
    const float* W;      // packed [Cin][KW][co_pad]
    const float* Wf;     // optional fragment-order copy of W (conv_pack_frag): small batches use it
    int wf_tap;          // Wf is in conv_pack_frag_tap's tap-major order (Cin = 512)
    const float* Wf16;   // optional conv_pack_frag_tap16 copy (with wf_tap): small grids take 16-channel tiles
    const float* scale;  // [Cout] (null = 1)
    const float* shift;  // [Cout] (null = 0)
    const float* resid;  // [B][Tmax][out_ld] or null: out = resid + y (CONV_HIGHWAY: the layer input)
    const int* T;        // [B] valid frames per sentence
    int Tmax, Cin, Cout, co_pad, act;
    int pool2;           // stage max(in[t], in[t+1]) with in[T_b] = 0: CBHG's ConstantPad1d([0, 1]) +
                         // MaxPool1d(2, stride 1) (layers/tacotron.py:137-139, 188) fused into the next conv
    int out_ld;          // row stride of out / resid in floats (0 = Cout)
    // optional split-K workspace (>= CONV_SPLITK_FLOATS floats): small launches (batch-1 postnet /
    // encoder: ~100 output tiles) split the input channels over up to 16 workgroups per tile and
    // reduce the partial sums in a second launch, in split order (deterministic)
    float* part;
    int Ttile;  // frames covered by output tiles (>= max T_b; 0 = Tmax): a caller whose buffers are
                // sized for a cap (postnet: max_decoder_steps + 20) passes the batch's longest sentence
    int in_tmax;  // frames per sentence of `in` (0 = Tmax) and of `resid` (res_tmax): the synthesis
    int res_tmax; // postnet reads the decoder's mel history in place (max_decoder_steps + 21 steps)
    int tmul;     // T[b] counts groups of tmul frames (0 = 1): the decoder's step counts, r frames each
    // optional [CONV_TICKETS] zeroed ints beside `part`: the split-K launch then reduces its own
    // partials (the last workgroup of each output tile; the words are left zero again)
    int* tickets;
};
constexpr size_t CONV_SPLITK_FLOATS = (size_t)1 << 20;  // split x tiles <= 1024 -> <= 1M partials
constexpr int CONV_TICKETS = 1024;                       // output tiles of one split-K launch

constexpr int CONV_BN = 64;  // output channels per tile
inline int conv_co_pad(int Cout) { return (Cout + CONV_BN - 1) / CONV_BN * CONV_BN; }

// W [Cout][Cin][KW] (PyTorch Conv1d layout) -> packed [Cin][KW][co_pad]
hipError_t conv_pack(const float* W, int Cout, int Cin, int KW, float* out, hipStream_t s);
// CBHG bank member W [Cout][Cin][k] into a KWmax-tap slab at channels [co_off, co_off + Cout):
// tap j lands on slot j + (KWmax-1)/2 - (k-1)/2, which reproduces the member's own
// ConstantPad1d([(k-1)/2, k/2]) (layers/tacotron.py:126-134) under the slab's centred window.
// The caller zeroes the slab first.
hipError_t conv_pack_bank(const float* W, int Cout, int Cin, int k, int KWmax, int co_off, int co_pad, float* out,
                          hipStream_t s);
// packed [K = Cin * KW][co_pad] -> the small-batch kernel's fragment order (K % 8 == 0, co_pad % 32 == 0)
hipError_t conv_pack_frag(const float* W, int K, int co_pad, float* out, hipStream_t s);
// the tap-major fragment order (k' = tap Cin + ci) of the small-batch conv's TAP form; Cin = 512 only
hipError_t conv_pack_frag_tap(const float* W, int Cin, int KW, int co_pad, float* out, hipStream_t s);
// the same for 16-column tiles (the small-batch conv's 16-channel form)
hipError_t conv_pack_frag_tap16(const float* W, int Cin, int KW, int co_pad, float* out, hipStream_t s);
bool conv_frag_tap_ok(int Cin);
// W [Cout][Cin] (Linear layout, rows stacked into Cout) -> packed [Cin][1][co_pad]
hipError_t linear_pack_as_conv(const float* W, int Cout, int Cin, int co_offset, int co_pad, float* out,
                               hipStream_t s);
// same, row n of W to packed column co_offset + n * stride (interleaved Highway H/T rows)
hipError_t linear_pack_strided(const float* W, int Cout, int Cin, int co_offset, int stride, int co_pad, float* out,
                               hipStream_t s);
// dst[i * stride] = src[i], i < n
hipError_t copy_strided(const float* src, int n, float* dst, int stride, hipStream_t s);
// scale = gamma / sqrt(var + eps); shift = beta + (bias - mean) * scale (bias may be null)
hipError_t fold_bn(const float* bias, const float* gamma, const float* beta, const float* mean, const float* var,
                   int C, float eps, float* scale, float* shift, hipStream_t s);
// KW in {1, 3, 5, 8, 16}; Cin must be a multiple of the K step (16 for KW <= 5, 8 for KW = 8, 4 for
// KW = 16).  frames_hint = sum of T_b picks the tile height (small batches: 16 frames).
hipError_t conv_launch(const ConvArgs& a, int KW, int B, int frames_hint, hipStream_t s);

}  // namespace tts
