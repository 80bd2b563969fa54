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
// Ping-pong buffers: row pointer = p + ((step + par) & 1) * pstride when par >= 0.
struct Seg {
    const float* p;
    int64_t pstride;
    int par;  // -1: no ping-pong
    int ld;   // row stride (floats)
    int len;  // multiple of 16
};

enum Epi { EPI_LINEAR = 0, EPI_LSTM = 1 };
// Decoder stage a launch serves; fixes the epilogue (LSTM roles use EPI_LSTM).
enum Role { ROLE_PRENET = 0, ROLE_ATT_LSTM = 1, ROLE_QUERY = 2, ROLE_DEC_LSTM = 3, ROLE_MEL = 4 };
enum Act { ACT_NONE = 0, ACT_RELU = 1 };

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
    const int* step;      // device step counter or null (=0)
    const int* done;      // per-row done flags or null
    const int* n_active;  // early exit when *n_active == 0, or null
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

}  // namespace tts
