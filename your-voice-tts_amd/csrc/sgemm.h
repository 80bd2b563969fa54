// Skinny fp32 GEMM for the decoder step: out[b][n] = epi(sum_k X[b][k] * W[n][k]), B <= 64.
//
// Weights are repacked once into MFMA-fragment order so that every weight load of a wave is
// one contiguous, perfectly coalesced 1 KiB (64 lanes x float4):
//   packed[((ntile*nchunks + c)*64 + lane)*4 + j] = W[ntile*16 + (lane&15)][c*16 + (lane>>4)*4 + j]
// A k-chunk of 16 feeds four v_mfma_f32_16x16x4_f32 (component j of every lane's float4 is
// k = c*16 + (lane>>4)*4 + j, the same permutation on both operands).  The activation rows
// (batch) are the MFMA M dimension, padded to 16 per m-tile.  K is split over the waves of a
// workgroup and reduced through LDS in a fixed order (deterministic).
#pragma once
#include "common.h"

namespace tts {

// One input segment of the logically concatenated activation row X[b] = [seg0 | seg1 | seg2].
// Pointers are bound per launch (the decoder captures one graph per step parity), so a launch
// can issue its activation loads before it reads the device step state.
struct Seg {
    const float* p;
    int ld;   // row stride (floats)
    int len;  // multiple of 16
    // fragment-order mirror of the same values (common.h: frag_idx with SGemmArgs::ntf m-tiles),
    // already offset to the segment's first chunk; when every segment has one the launch reads
    // the mirrors (sgemm_launch: the batched 4-wave kernel)
    const float* pf = nullptr;
};

enum Epi { EPI_LINEAR = 0, EPI_LSTM = 1, EPI_MEL_FUSED = 2, EPI_ENC_LSTM = 3, EPI_GRU = 4 };

// EPI_GRU: torch GRUCell (gate rows r, z, n; ATen's h' = (h - n) * z + n) for the Tacotron decoder
// (layers/tacotron.py:289, 304-305, 370-381).  A 16-row tile holds, for 4 hidden units u
// (ROWMAP_GRU), [W_ir x + W_hr h | W_iz x + W_hz h | W_in x | W_hn h], so that
// n = tanh(W_in x + b_in + r * (W_hn h + b_hn)) keeps its two halves apart.  Optional residual
// output dout = h' + res (the decoder GRU stack's residual connection, :380-381).
struct GruEpi {
    const float* h;  // previous hidden state [b * ldh + unit]
    int ldh;
    const float* res;  // residual input [b * ldr + unit] or null
    int ldr;
    float* dout;  // h' + res, or null
    int ldd;
};

// EPI_ENC_LSTM: one step s of the bidirectional encoder LSTM (layers/tacotron2.py:56-61, 82):
// workgroups [0, tiles_per_dir) run the forward direction on seg[0] = h_fwd(s-1) at position s,
// the rest the reverse direction on seg[1] = h_bwd(s-1) at position L_b-1-s.  Gates add the
// precomputed input projection xi (both biases folded in); sentences with s >= L_b are idle.
struct EncLstm {
    int tiles_per_dir;
    int H;
    int s;
    const int* lens;
    const float* xi;  // [B][Tmax][2*4H]
    int Tmax;
    float* c;         // [2][cstride]
    int64_t cstride;  // per-direction stride of c and h_next (>= B*H)
    float* h_next;    // [2][cstride]
    float* enc_out;   // [B][Tmax][2H]
};
// Decoder stage a launch serves; fixes the epilogue (LSTM roles use EPI_LSTM, ROLE_MEL_FUSED
// uses EPI_MEL_FUSED).
enum Role {
    ROLE_PRENET = 0, ROLE_ATT_LSTM = 1, ROLE_QUERY = 2, ROLE_DEC_LSTM = 3, ROLE_MEL = 4, ROLE_MEL_FUSED = 5,
    ROLE_ENC_LSTM = 6,
    // Tacotron / TacotronGST decoder step (tacotron_api.hip)
    ROLE_T_PRENET1 = 7, ROLE_T_PRENET2 = 8, ROLE_T_ATT_GRU = 9, ROLE_T_QUERY = 10, ROLE_T_PROJ = 11,
    ROLE_T_DEC_GRU = 12, ROLE_T_MEL = 13, ROLE_T_PRE1_STOP = 14
};
enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_SIGMOID = 2 };

// EPI_MEL_FUSED: one GEMM over x = [h_dec | ctx] whose output rows are
//   [0, nmel)            mel frame(s)                  -> history
//   [nmel, nmel+256)     prenet layer-1 pre-activation -> relu -> pre1 (next step's prenet)
//   nmel+256             stop-token logit              -> sigmoid -> history + stop rule
// using weights folded at load time: W1' = W1 W_mel, w_stop' = [w_s_h | 0] + w_s_mel W_mel.
// The Tacotron decoder uses it with nmel = 0 over x = [mel out | decoder out] (its mel has a
// sigmoid, so nothing folds): rows [0, 256) = [W1 | 0], row 256 = the stopnet, rule = 1.
struct MelFused {
    int nmel;
    float* pre1;
    int ldp;
    float* stop_hist;
    int64_t stop_ldb;
    const int* lens;
    const float* tail;
    int* flag1;
    int* count;
    int* done;
    int* n_steps;
    int* state_next;  // int2 {t+1, n_active} read by the next step (other parity slot)
    int* stop_acc;    // zero at rest: the row groups' active counts meet here (grid.y > 1)
    float* pre1f;     // fragment mirror of pre1 (SGemmArgs::ntf m-tiles) or null
    int max_steps;
    int rule;  // 0: Tacotron2 stop rule (layers/tacotron2.py:267-277); 1: Tacotron (layers/tacotron.py:464-469);
               // 2: teacher forcing (Decoder.forward, layers/tacotron2.py:227-247): no rule, stop logits
};

struct SGemmArgs {
    Seg seg[3];
    int nseg;
    const float* W;  // packed
    int K, N, B;
    const float* bias;  // logical row order, may be null
    int act;
    float* out;
    int64_t out_pstride;
    int out_par;
    int ldo;
    float* out2;  // optional plain copy of the output rows
    int ldo2;
    // optional fragment-order mirror of the output (frag_idx(b, outf_k0 + column, ntf)); ntf is
    // also the m-tile count of the input mirrors (Seg::pf)
    float* outf;
    int outf_k0;
    int ntf;
    float* hist;  // optional history: hist[b*ldh + step*N + n] for active rows, step < hist_cap
    int64_t ldh;
    int hist_cap;
    float* cell;  // LSTM cell state [b*ldc + unit], updated in place
    int ldc;
    const int* step;      // int2 {step, n_active} of this step's parity slot, or null (= {0, 1});
                          // the kernel exits early when n_active == 0
    const int* done;      // per-row done flags or null
    const int* n_active;  // unused (kept adjacent to step)
    MelFused mf;          // EPI_MEL_FUSED only
    EncLstm enc;          // EPI_ENC_LSTM only
    GruEpi gru;           // EPI_GRU only
};

// Row maps used when repacking reference matrices.
enum RowMap { ROWMAP_IDENTITY = 0, ROWMAP_LSTM = 1, ROWMAP_GRU = 2 };

// Repack [A (N x K1) | B (N x K2)] (row-major, fp32, reference layout) into fragment order.
// ROWMAP_LSTM: logical row ntile*16 + gate*4 + u  <-  reference row gate*H + ntile*4 + u.
// ROWMAP_GRU (N = 4H, A = W_ih [3H][K1], B = W_hh [3H][K2]): logical gate g of unit
// ntile*4 + u is [W_ir | W_hr], [W_iz | W_hz], [W_in | 0], [0 | W_hn] for g = 0..3; biases
// b_ir + b_hr, b_iz + b_hz, b_in, b_hn.
hipError_t sgemm_pack(const float* A, int K1, const float* Bm, int K2, int N, int rowmap, int H,
                      float* packed, hipStream_t s);
// Logical-order bias: bias_l[n_l] = a[row(n_l)] (+ b[row(n_l)] if b), rows >= N are zero.
hipError_t sgemm_pack_bias(const float* a, const float* b, int N, int rowmap, int H, float* out,
                           hipStream_t s);
inline size_t sgemm_packed_floats(int N, int K) { return (size_t)((N + 15) / 16) * 16 * K; }

hipError_t sgemm_launch(const SGemmArgs& a, int role, hipStream_t s);
// Wf [nmel+257][K] logical rows + bf [nmel+257] for ROLE_MEL_FUSED (see MelFused).
hipError_t fold_mel_weights(const float* Wm, const float* bm, const float* W1, const float* b1, const float* ws,
                            const float* bs, int nmel, int K, int hdec, float* Wf, float* bf, hipStream_t s);
// Eval-mode BatchNorm1d after a linear layer (LinearBN, common_layers.py:28-52) folded into it:
// Wout = diag(s) W, bout = s (b - mean) + beta, s = gamma / sqrt(var + eps) (fp64, rounded once);
// b may be null (bias=False).  W, Wout: [rows][cols] reference layout.
hipError_t fold_linear_bn(const float* W, const float* b, const float* gamma, const float* beta, const float* mean,
                          const float* var, int rows, int cols, float eps, float* Wout, float* bout, hipStream_t s);

}  // namespace tts
