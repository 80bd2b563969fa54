// Decoder-step state and the non-GEMM kernels of the step (init, processed inputs, attention).
#pragma once
#include "common.h"

namespace tts {

constexpr int ENC = 512;   // encoder embedding dim (layers/tacotron2.py:104)
constexpr int HATT = 1024; // attention_rnn_dim
constexpr int HDEC = 1024; // decoder_rnn_dim
constexpr int PRE = 256;   // prenet_dim
constexpr int ADIM = 128;  // attention_dim
constexpr int NLOC = 32;   // location filters
constexpr int KLOC = 31;   // location kernel
constexpr int XA = PRE + ENC;  // [prenet | ctx] row of the attention-LSTM input
constexpr int ATT_THREADS = 1024;  // one thread per encoder position (L <= 1024)
constexpr int ATT_WAVES = ATT_THREADS / 64;
constexpr int ATT_SPLIT = 4;  // workgroups per sentence of the general attention launch with epart

// Flags (tts_decoder_config) + weights + device state pointers, passed by value.
struct AttnArgs {
    int attn_norm, forward_attn, trans_agent, forward_attn_mask, location_attn, windowing;
    int Lcap;  // row stride of per-position arrays
    int B;
    int enc_dim;    // encoder width: 512 (Tacotron2) or 256 (Tacotron / TacotronGST, query width 256)
    int ctx_ld;     // row stride of ctx (XA for Tacotron2)
    int tail_rule;  // 0: tail = w[L-2] + w[L-1] (layers/tacotron2.py:268); 1: w[L-1] (layers/tacotron.py:465)
    // weights (reference layout)
    const float* v;        // [128]
    const float* v_b;      // [1]
    const float* ta_w;     // [enc_dim + query width] = [ctx | h_att]
    const float* ta_b;     // [1]
    const float* loc_conv; // [32][2][31]
    const float* loc_dense;// [128][32]
    // inputs
    const float* q;        // [B][128] processed query (unused when wqT is set)
    const float* wqT;      // attention_kernel: [HATT_][128] query_layer weight, transposed, or null:
                           // then the kernel computes the processed query itself from h_att
    const float* Pt;       // [B][128][Lcap] processed inputs, transposed
    const float* enc;      // [B][Lcap][enc_dim]
    const int* lens;       // [B]
    const float* h_att;    // [B][query width] this step's attention-RNN output
    const float* epart;    // [B][ADIM/16][Lcap] energy partials from query_energy_kernel (Tacotron2: every
                           // attention configuration; null: attention_kernel evaluates the energies)
    float* locf;           // with epart and location_attn: [B][NLOC][Lcap] the NEXT step's location
                           // features (location_conv over [att_w; att_cum]), written at the step's end
    // with epart (ATT_SPLIT workgroups per sentence, each recomputing the weights): alpha, att_cum
    // ([2][B][Lcap]) and nidx, win_idx ([2][B]) by step parity, slot strides sstride / istride (the
    // step reads slot t & 1 and writes the other); the transition agent's u from the previous
    // step's context and attention-RNN output (ctx rows of stride ctx_ld, h rows of HATT)
    int64_t sstride;
    int istride;
    const float* ctx_prev;
    const float* h_att_prev;
    // state
    float* alpha;          // [B][Lcap]
    float* att_w;          // [B][Lcap]
    float* att_cum;        // [B][Lcap]
    float* u;              // [B]
    int* win_idx;          // [B]
    int* nidx;             // [B] argmax of prev_alpha for the next step (forward mask)
    float* tail;           // [B] att_w[L-2] + att_w[L-1]
    // outputs
    float* ctx;            // [B] rows of stride ctx_ld: context written to ctx[b*ctx_ld + d]
    float* ctxf;           // fragment mirror (frag_idx(b, ctxf_k0 + d, ntf)) or null
    int ctxf_k0, ntf;
    float* align_hist;     // [B][hist_cap][Lalign] or null
    int64_t align_ldb;     // stride per sentence
    int Lalign;
    int hist_cap;
    const int* step;       // int2 {step, n_active} of this step's parity slot
    const int* done;
};

struct InitArgs {
    int B, Lcap, nmel;
    int keep;  // continuous mode: keep h / c / context / memory, restart attention and stop state
    const int* lens;
    const float* att_init;  // [1024]
    const float* dec_init;  // [1024]
    const float* go;        // [nmel]
    float* h_att; int64_t h_pstride;
    float* c_att;
    float* h_dec;
    float* c_dec;
    float* xa; int64_t xa_pstride;
    float* mem;
    float* alpha; float* att_w; float* att_cum; float* u; int* win_idx; int* nidx; float* tail;
    int* flag1; int* count; int* done; int* n_steps; int* step; int* n_active;
    float* locf;  // [B][NLOC][Lcap] step-0 location features (zero attention state: zeros), or null
    // batch-1 resident runs: the cached go-frame prenet row copied into pre1 (null: the prenet GEMM
    // runs), and a granule array zeroed by INIT_ZERO_BLOCKS extra workgroups (null: none)
    const float* pre1_go; float* pre1;
    unsigned long long* zero; int nzero;
};
constexpr int INIT_ZERO_BLOCKS = 16;

// Processed query + energy partials (one workgroup per (16 attention dims, sentence)):
//   q[b][d] = W_q h_att[b]  (query_layer, common_layers.py:170/179)
//   epart[b][tile][j] = sum_{d in tile} v[d] tanh(q[b][d] + P[b][j][d])  (get_attention, :178-182)
// The attention launch sums the ADIM/16 partials per position instead of evaluating 128 tanh
// per position on one compute unit.
constexpr int QE_TILES = ADIM / 16;
struct QEArgs {
    const float* Wq;    // sgemm-packed W_q [QE_TILES][HATT/16 chunks][64 lanes][4]
    const float* h;     // [B][HATT] h_att_t
    const float* v;     // [ADIM]
    const float* Pt;    // [B][ADIM][Lcap]
    const int* lens;
    int Lcap;
    int energies;       // 0: q only (the general attention kernel evaluates the energies itself)
    const float* locf;       // [B][NLOC][Lcap] this step's location features, or null (no location layer)
    const float* loc_dense;  // [ADIM][NLOC] location_dense weight (with locf)
    float* q;           // [B][ADIM]
    float* epart;       // [B][QE_TILES][Lcap]
    const int* step;    // int2 {step, n_active}
};
hipError_t launch_query_energy(const QEArgs& a, int B, hipStream_t s);
bool attention_uses_epart(const AttnArgs& a);

hipError_t launch_decoder_init(const InitArgs& a, hipStream_t s);
// launch_project_inputs (ENC = 512) and launch_decoder_init as one launch
hipError_t launch_project_init(const float* enc, const float* W, int B, int Lmax, int Lcap, float* Pt, const InitArgs& ia,
                               hipStream_t s);
// teacher forcing: mem[b] = teacher row step-1 of frames[b] (ldb floats per sentence), go frame at step 0
hipError_t launch_teacher_memory(const float* frames, int64_t ldb, int width, const int* step, float* mem, int B,
                                 hipStream_t s);
hipError_t launch_zero_tail(float* dst, int64_t ldb, const int* n_steps, int width, int nmax, int B, hipStream_t s);
// enc_dim 512 (Tacotron2) or 256 (Tacotron / TacotronGST)
hipError_t launch_project_inputs(const float* enc, const float* W, int B, int Lmax, int Lcap, float* Pt, hipStream_t s,
                                 int enc_dim = ENC);
hipError_t launch_attention(const AttnArgs& a, hipStream_t s);
hipError_t transpose_f32(const float* src, int rows, int cols, float* dst, hipStream_t s);  // dst[c][r] = src[r][c]
size_t attention_smem_bytes(int Lcap, int location);
hipError_t attention_prepare(int Lcap, int location);  // raise the dynamic-LDS limit once

}  // namespace tts
