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
};

enum Epi { EPI_LINEAR = 0, EPI_LSTM = 1, EPI_MEL_FUSED = 2, EPI_ENC_LSTM = 3 };

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
    ROLE_ENC_LSTM = 6
};
enum Act { ACT_NONE = 0, ACT_RELU = 1 };

// EPI_MEL_FUSED: one GEMM over x = [h_dec | ctx] whose output rows are
//   [0, nmel)            mel frame(s)                  -> history
//   [nmel, nmel+256)     prenet layer-1 pre-activation -> relu -> pre1 (next step's prenet)
//   nmel+256             stop-token logit              -> sigmoid -> history + stop rule
// using weights folded at load time: W1' = W1 W_mel, w_stop' = [w_s_h | 0] + w_s_mel W_mel.
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
    int max_steps;
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
};

// Row maps used when repacking reference matrices.
enum RowMap { ROWMAP_IDENTITY = 0, ROWMAP_LSTM = 1 };

// Repack [A (N x K1) | B (N x K2)] (row-major, fp32, reference layout) into fragment order.
// ROWMAP_LSTM: logical row ntile*16 + gate*4 + u  <-  reference row gate*H + ntile*4 + u.
hipError_t sgemm_pack(const float* A, int K1, const float* Bm, int K2, int N, int rowmap, int H,
                      float* packed, hipStream_t s);
// Logical-order bias: bias_l[n_l] = a[row(n_l)] (+ b[row(n_l)] if b), rows >= N are zero.
hipError_t sgemm_pack_bias(const float* a, const float* b, int N, int rowmap, int H, float* out,
                           hipStream_t s);
inline size_t sgemm_packed_floats(int N, int K) { return (size_t)((N + 15) / 16) * 16 * K; }

hipError_t sgemm_launch(const SGemmArgs& a, int role, hipStream_t s);
// Wf [nmel+257][K] logical rows + bf [nmel+257] for ROLE_MEL_FUSED (see MelFused).
hipError_t fold_mel_weights(const float* Wm, const float* bm, const float* W1, const float* ws, const float* bs,
                            int nmel, int K, int hdec, float* Wf, float* bf, hipStream_t s);

}  // namespace tts
