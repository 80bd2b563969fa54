// Microbenchmark (measurement only): cost of one all-to-all hand-off edge of the resident decoder
// (256 workgroups x 512 threads, one per CU; 8-byte {tag, value} granules), repeated R rounds
// (round r+1 is published only after round r is fully gathered).
//   mode 0: flat      — every CU publishes 4 granules device-wide (sc1), GW waves sweep all 1024
//   mode 1: two-level — every CU polls its XCD rank's 32-granule slice device-wide (one wave),
//                       republishes it XCD-locally (sc0), then GW waves sweep the XCD's 1024 copies
//   mode 2: XCD-local — every CU publishes 8 granules XCD-locally, GW waves sweep the XCD's 256
//   mode 3: flat 8 KB, only the 32 CUs of one rank-class read (the other CUs publish and skip)
//   mode 4: flat device-wide 1024 granules as 16-byte pairs; mode 5: XCD-local 256 as pairs
// usage: edge <mode> <GW> <rounds> [first_sleep]: first_sleep x s_sleep 4 before a round's first
// poll (round 6: a poll storm from every CU slows the stores it waits for).  Every spin is bounded
// (1 << 22 polls): a lost round ends the kernel with a wrong time instead of a hang.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned long long u64;
typedef __attribute__((address_space(1))) u64 gu64;

__device__ __forceinline__ void pub_dev(u64* g, unsigned tag, float v) {
    __hip_atomic_store((gu64*)g, ((u64)tag << 32) | (u64)__float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void pub_xcd(u64* g, unsigned tag, float v) {
    __hip_atomic_store((gu64*)g, ((u64)tag << 32) | (u64)__float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ u64 peek(u64* g) {
    return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int N, typename F>
__device__ __forceinline__ void sweep(u64* g, unsigned tag, float (&v)[N], F idx) {
    for (int spin = 0; spin < (1 << 22); ++spin) {
        bool ok = true;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const int k = idx(i);
            if (k >= 0) {
                const u64 x = peek(g + k);
                v[i] = __uint_as_float((unsigned)x);
                ok = ok && (unsigned)(x >> 32) == tag;
            }
        }
        if (__all(ok)) return;
    }
}

typedef __attribute__((ext_vector_type(2))) unsigned long long u64x2;
typedef __attribute__((address_space(1))) u64x2 gu64x2;
// N 16-byte loads per lane, each = granules (2k, 2k + 1) of pair index k = idx(i)
template <int N, typename F>
__device__ __forceinline__ void sweep16(u64* g, unsigned tag, float (&v)[2 * N], F idx) {
    for (int spin = 0; spin < (1 << 22); ++spin) {
        bool ok = true;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const int k = idx(i);
            if (k >= 0) {
                u64x2 x;
                asm volatile("global_load_dwordx4 %0, %1, off sc1\n s_waitcnt vmcnt(0)" : "=v"(x) : "v"((gu64x2*)(g + 2 * k)) : "memory");
                v[2 * i] = __uint_as_float((unsigned)x.x);
                v[2 * i + 1] = __uint_as_float((unsigned)x.y);
                ok = ok && (unsigned)(x.x >> 32) == tag && (unsigned)(x.y >> 32) == tag;
            }
        }
        if (__all(ok)) return;
    }
}

constexpr int GR_TAB = 0, GR_DEV = 512, GR_X = GR_DEV + 2 * 1024, GR_TOTAL = GR_X + 2 * 8 * 1024;

template <int GW>
__global__ __launch_bounds__(512, 1) void edge_kernel(u64* gran, int mode, int rounds, float* sink, long long* ticks,
                                                      int first_sleep) {
    const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ float xs[1024];
    __shared__ int info[4];
    int xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 7;
    if (tid == 0) pub_dev(gran + GR_TAB + c, 1u, __int_as_float(xcc));
    if (wave == 0) {
        float v4[4];
        sweep<4>(gran + GR_TAB, 1u, v4, [&](int i) { return lane * 4 + i; });
        int rank = 0;
        for (int i = 0; i < 4; ++i) {
            const int x = __float_as_int(v4[i]) & 7;
            rank += __popcll(__ballot(x == xcc && lane * 4 + i < c));
        }
        if (lane == 0) info[0] = rank;
    }
    __syncthreads();
    const int rank = info[0];
    float acc = 0.f;
    const long long t0 = wall_clock64();
    for (int r = 0; r < rounds; ++r) {
        const unsigned tag = 2u + (unsigned)r;
        const int par = r & 1;
        u64* gd = gran + GR_DEV + par * 1024;
        u64* gx = gran + GR_X + (par * 8 + xcc) * 1024;
        if (mode == 0 || mode == 1 || mode == 3 || mode == 4) {
            if (tid < 4) pub_dev(gd + 4 * c + tid, tag, acc + (float)tid);
        } else {
            if (tid < 8) pub_xcd(gx + 8 * rank + tid, tag, acc + (float)tid);
        }
        if (mode == 1 && wave == 0) {
            // relay: this CU's 32-granule slice of the device-wide vector, XCD-locally
            float v1[1];
            sweep<1>(gd, tag, v1, [&](int) { return lane < 32 ? rank * 32 + lane : -1; });
            if (lane < 32) pub_xcd(gx + rank * 32 + lane, tag, v1[0]);
        }
        if (mode == 3 && (rank & 7) != 0) {
            __syncthreads();
            continue;
        }
        if (wave < GW)
            for (int i = 0; i < first_sleep; ++i) __builtin_amdgcn_s_sleep(4);
        if (mode >= 4 && wave < GW) {
            // 16-byte pair loads: mode 4 flat device-wide, mode 5 XCD-local 256
            constexpr int PER = 512 / (64 * GW);  // pairs per lane
            const int n = mode == 5 ? 128 : 512;
            float v[2 * (PER > 0 ? PER : 1)];
            u64* src = mode == 4 ? gd : gx;
            sweep16<(PER > 0 ? PER : 1)>(src, tag, v, [&](int i) {
                const int k = wave * 64 * PER + i * 64 + lane;
                return k < n ? k : -1;
            });
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                xs[2 * (wave * 64 * PER + i * 64 + lane)] = v[2 * i];
                xs[2 * (wave * 64 * PER + i * 64 + lane) + 1] = v[2 * i + 1];
            }
        } else if (wave < GW) {
            constexpr int PER = 1024 / (64 * GW);
            const int n = mode == 2 ? 256 : 1024;
            float v[PER];
            u64* src = mode == 0 || mode == 3 ? gd : gx;
            sweep<PER>(src, tag, v, [&](int i) {
                const int k = wave * 64 * PER + i * 64 + lane;
                return k < n ? k : -1;
            });
#pragma unroll
            for (int i = 0; i < PER; ++i) xs[wave * 64 * PER + i * 64 + lane] = v[i];
        }
        __syncthreads();
        acc += xs[(tid * 7 + r) & 1023] * 1e-30f;
    }
    const long long t1 = wall_clock64();
    if (tid == 0) {
        sink[c] = acc;
        ticks[c] = t1 - t0;
    }
}

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0, gw = argc > 2 ? atoi(argv[2]) : 4,
              rounds = argc > 3 ? atoi(argv[3]) : 2000, first_sleep = argc > 4 ? atoi(argv[4]) : 0;
    u64* gran;
    float* sink;
    long long* ticks;
    (void)hipMalloc(&gran, sizeof(u64) * GR_TOTAL);
    (void)hipMalloc(&sink, 4 * 256);
    (void)hipMalloc(&ticks, 8 * 256);
    int rate = 0;
    (void)hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);
    auto fn = gw == 8 ? (void*)edge_kernel<8> : gw == 2 ? (void*)edge_kernel<2> : (void*)edge_kernel<4>;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipMemset(gran, 0, sizeof(u64) * GR_TOTAL);
        void* args[] = {&gran, (void*)&mode, (void*)&rounds, &sink, &ticks, (void*)&first_sleep};
        (void)hipLaunchKernel(fn, dim3(256), dim3(512), args, 0, 0);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("fail\n");
            return 1;
        }
        std::vector<long long> t(256);
        (void)hipMemcpy(t.data(), ticks, 8 * 256, hipMemcpyDeviceToHost);
        long long mx = 0;
        for (long long v : t) mx = v > mx ? v : mx;
        printf("mode %d GW %d rounds %d first_sleep %d: %.3f us per round\n", mode, gw, rounds, first_sleep,
               1e3 * (double)mx / rate / rounds);
    }
    return 0;
}
