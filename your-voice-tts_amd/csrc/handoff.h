// In-launch hand-offs of the resident (persistent) decoders: 8-byte {tag:32 | fp32} granules
// published with relaxed atomic stores and polled with L1-bypassing loads (MI355X_MICROARCH.md
// "Valid forms": the fence-free hand-off).  Shared by resident_decoder.hip (batch 1) and
// resident_batch.hip (batches of 2-8).
#pragma once
#include <hip/hip_runtime.h>

namespace tts {
namespace handoff {

typedef unsigned long long u64;
typedef __attribute__((address_space(1))) u64 gu64;
typedef __attribute__((address_space(1))) int gint;

#ifndef RES_SLEEP
#define RES_SLEEP 0  // s_sleep between polls: 0 measured 11.03 -> 10.70 us per step (tools/dec_ab.sh)
#endif

__device__ __forceinline__ void publish(u64* g, unsigned tag, float v) {
    __hip_atomic_store((gu64*)g, ((u64)tag << 32) | (u64)__float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
// Same-XCD hand-off: a workgroup-scope store (global_store ... sc0) keeps the line in the XCD's
// L2, which every CU of that XCD reads with the agent-scope (sc1, L1-bypassing) loads of sweep().
__device__ __forceinline__ void publish_xcd(u64* g, unsigned tag, float v) {
    __hip_atomic_store((gu64*)g, ((u64)tag << 32) | (u64)__float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ u64 peek(u64* g) {
    return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The first failure of a launch wins (the other workgroups then time out in cascade); its step
// and workgroup go to status[1], status[2] (diagnostics).
__device__ __forceinline__ void fail(int* status, int code, int step = -1) {
    int expected = 0;
    if (__hip_atomic_compare_exchange_strong((gint*)status, &expected, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store((gint*)status + 1, step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store((gint*)status + 2, (int)blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// One wave polls its N granules per lane (idx(i) < 0: none) until every tag equals tag(i);
// false after `tmo` wall-clock ticks (the caller flags the error, the grid drains).
template <int N, typename F, typename T>
__device__ __forceinline__ bool sweep2(u64* g, F idx, T tag, float (&v)[N], long long tmo) {
    long long t_end = 0;
    for (int spin = 0;; ++spin) {
        bool ok = true;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const int k = idx(i);
            if (k >= 0) {
                const u64 x = peek(g + k);
                v[i] = __uint_as_float((unsigned)x);
                ok = ok && (unsigned)(x >> 32) == tag(i);
            }
        }
        if (__all(ok)) return true;
        if (spin == 0) {
            t_end = (long long)wall_clock64() + tmo;
        } else if ((spin & 31) == 0 && (long long)wall_clock64() > t_end) {
            return false;
        }
        if (RES_SLEEP) __builtin_amdgcn_s_sleep(RES_SLEEP);
    }
}
// One wave polls its N granules per lane (idx(i) < 0: none) until every tag equals `tag`;
// false after `tmo` wall-clock ticks (the caller flags the error, the grid drains).
template <int N, typename F>
__device__ __forceinline__ bool sweep(u64* g, unsigned tag, float (&v)[N], F idx, long long tmo) {
    return sweep2<N>(g, idx, [&](int) { return tag; }, v, tmo);
}

// Granule pairs: every gather of the step loop reads ONE 16-byte pair (2 granules) per lane, an
// sc1 buffer load (L1-bypassing; volatile, so every poll re-issues it).  A poll's latency grows
// with the loads per lane (tools/microbench/edge.hip, round 4: device-wide 1024 granules 2.31 us per
// edge with 4 x 8-byte loads per lane on 4 waves, 1.60-1.63 with one pair or two granules per lane
// on 8 waves; XCD-local 256 granules 1.14 us with 4 per lane on one wave, 0.47 with one pair per
// lane on 2 waves).  Each 8-byte half is written whole by one store, so a pair is never torn
// within a half (MI355X_MICROARCH.md "Valid forms", R2's granule); both tags are checked.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int SC1_VOLATILE = (int)0x80000010u;  // buffer aux: sc1 (bit 4) | volatile (bit 31)
constexpr int VOLATILE_AUX = (int)0x80000000u;  // buffer aux: volatile only (default cache policy)
constexpr int OOB_OFF = 0x7FFFFFF0;             // past every buffer: reads 0, no access
// One wave polls one pair per lane at granule slot `slot` (even; < 0: none) until its tags equal
// `tag` (the second half only when `both`); v0/v1 = the two values.  false after `tmo` ticks.
__device__ __forceinline__ bool sweep_pair(__amdgpu_buffer_rsrc_t r, int slot, bool both, unsigned tag, float& v0,
                                           float& v1, long long tmo) {
    long long t_end = 0;
    for (int spin = 0;; ++spin) {
        bool ok = true;
        if (slot >= 0) {
            const u32x4 x = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, slot * 8, 0, SC1_VOLATILE));
            v0 = __uint_as_float(x.x);
            v1 = __uint_as_float(x.z);
            ok = x.y == tag && (!both || x.w == tag);
        }
        if (__all(ok)) return true;
        if (spin == 0) {
            t_end = (long long)wall_clock64() + tmo;
        } else if ((spin & 31) == 0 && (long long)wall_clock64() > t_end) {
            return false;
        }
        if (RES_SLEEP) __builtin_amdgcn_s_sleep(RES_SLEEP);
    }
}

}  // namespace handoff
}  // namespace tts
