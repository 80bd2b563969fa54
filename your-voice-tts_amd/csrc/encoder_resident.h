// Resident batch-1 encoder BiLSTM (see encoder_resident.hip).
#pragma once
#include "common.h"

namespace tts {

constexpr int ENC_RES_STATUS_PLACEMENT = 50;  // fewer than the roles' workgroups on the XCD(s) they take

struct EncResArgs {
    const float4* w;     // packed W_hh of both directions (encoder_resident_pack)
    const float* xi;     // [Tmax][2][1024] input projection + both biases (sentence 0)
    int L;               // encoder length of the sentence
    int64_t hdir;        // per-direction stride of h0 / c0 / h_fin / c_fin (floats)
    const float* h0;     // [2][hdir] initial h (forward, backward) or null (zeros)
    const float* c0;     // [2][hdir] initial c or null
    float* h_fin;        // [2][hdir] h_n
    float* c_fin;        // [2][hdir] c_n
    float* out;          // [Tmax][512] outputs (rows >= L untouched)
    unsigned long long* gran;  // encoder_resident_granules() u64, zeroed before every launch
    int* status;         // 0 ok; ENC_RES_STATUS_PLACEMENT; else a wait timed out
    long long tmo;       // wall_clock64 ticks per wait
    int first_sleep;     // s_sleep(1) count before a step's first h poll (TTS_ENC_FIRST_SLEEP)
    unsigned salt;       // per-launch tag salt (18 bits): launched directly, never from a graph,
                         // so no granule (or stale cache line) of an earlier launch can match
};

// Batched form (2 <= B <= 64, sentences at their own lengths, zero initial state): every XCD runs
// one direction (xcc & 1) for one group of up to 16 sentences (xcc >> 1), its 32 workgroups each
// holding 8 hidden units' W_hh rows as MFMA operands in registers; the step's h all-gather stays
// inside the XCD.  Needs >= 32 workgroups on every XCD (else status ENC_RES_STATUS_PLACEMENT).
struct EncResBatchArgs {
    const float* whh;    // [2][1024][256] W_hh (reference layout, forward then reverse)
    const float* xi;     // [B][Tmax][2][1024] input projection + both biases
    const int* lens;     // [B]
    int B, Tmax;
    float* out;          // [B][Tmax][512]
    unsigned long long* gran;  // encoder_resident_batch_granules() u64
    int* status;         // salt << 8 | code on failure (res_status_code)
    long long tmo;
    unsigned salt;
};
size_t encoder_resident_batch_granules();  // includes the trailing status word
hipError_t launch_encoder_resident_batch(const EncResBatchArgs& a, hipStream_t s, bool* launched);

size_t encoder_resident_weight_float4();
size_t encoder_resident_granules();  // includes the trailing status word
hipError_t encoder_resident_pack(const float* whh_fwd, const float* whh_bwd, float4* out, hipStream_t s);
// co-residency guaranteed or nothing launched (*launched = false): common.h launch_persistent
hipError_t launch_encoder_resident(const EncResArgs& a, hipStream_t s, bool* launched);

}  // namespace tts
