// Error reporting shared by every entry point of libtts_hip.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "common.h"

namespace tts {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

tts_status hip_fail(hipError_t e, const char* what, const char* file, int line) {
    char buf[512];
    std::snprintf(buf, sizeof(buf), "HIP error %d (%s) in %s at %s:%d", (int)e, hipGetErrorString(e), what, file, line);
    g_last_error = buf;
    return TTS_ERR_HIP;
}

int usable_cus() {
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    const char* cap = std::getenv("TTS_CU_CAP");
    if (cap && cap[0]) {
        const int c = std::atoi(cap);
        if (c >= 0 && c < ncu) ncu = c;
    }
    return ncu;
}

// Co-residency of a persistent grid: the occupancy of `fn` at this block size (queried once per
// kernel and cached: the query costs tens of microseconds) times the usable CUs must cover the
// grid, else the caller falls back.  The launch itself is a plain one by default; the kernels'
// waits are bounded and report a grid that still failed to become resident (another process
// holding CUs), which the callers turn into their fallback or an error.  TTS_COOP=1 launches with
// hipLaunchCooperativeKernel instead (the runtime's own guarantee; measured ~30 us per launch on
// this ROCm, ~2.5% of a configs[1] sentence over its three persistent launches).
hipError_t launch_persistent(const void* fn, dim3 grid, dim3 block, void** args, size_t smem, hipStream_t s,
                             bool* launched) {
    *launched = false;
    const long long blocks = (long long)grid.x * grid.y * grid.z;
    const int threads = (int)(block.x * block.y * block.z);
    struct Key {
        const void* fn;
        int threads;
        size_t smem;
    };
    static std::mutex mu;
    static std::vector<std::pair<Key, int>> cache;
    static const bool coop = [] {
        const char* c = std::getenv("TTS_COOP");
        return c && c[0] == '1';
    }();
    int per_cu = -1;
    {
        std::lock_guard<std::mutex> lk(mu);
        for (const auto& kv : cache)
            if (kv.first.fn == fn && kv.first.threads == threads && kv.first.smem == smem) per_cu = kv.second;
        if (per_cu < 0) {
            hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, smem);
            if (e != hipSuccess) return e;
            cache.push_back({Key{fn, threads, smem}, per_cu});
        }
    }
    // cannot be co-resident: fall back (TTS_CU_CAP is read per call: tests set it)
    if ((long long)per_cu * usable_cus() < blocks) return hipSuccess;
    hipError_t e;
    if (coop) {
        e = hipLaunchCooperativeKernel(fn, grid, block, args, (unsigned)smem, s);
        if (e == hipErrorCooperativeLaunchTooLarge) {
            (void)hipGetLastError();  // refused before anything ran: fall back
            return hipSuccess;
        }
    } else {
        e = hipLaunchKernel(fn, grid, block, args, smem, s);
    }
    if (e == hipSuccess) *launched = true;
    return e;
}

// The runtime's stream / event synchronize blocks on an interrupt once its short active wait
// expires: after a multi-millisecond persistent launch the host woke 35-50 us after the GPU went
// idle (configs[1] timeline, round 3), and the next stage's launches waited for it.  This records
// `ev` on `s` and polls it instead (one host core busy for the wait), falling back to the blocking
// wait after TTS_SPIN_MS milliseconds (default 200; 0 = always block).
hipError_t spin_sync(hipStream_t s, hipEvent_t ev) {
    hipError_t e = hipEventRecord(ev, s);
    if (e != hipSuccess) return e;
    return spin_wait(ev);
}

hipError_t spin_wait(hipEvent_t ev) {
    static const long long spin_ns = [] {
        const char* v = std::getenv("TTS_SPIN_MS");
        return (long long)((v && v[0]) ? std::atof(v) * 1e6 : 200e6);
    }();
    hipError_t e = hipSuccess;
    if (spin_ns > 0) {
        const auto t0 = std::chrono::steady_clock::now();
        for (unsigned k = 0;; ++k) {
            e = hipEventQuery(ev);
            if (e != hipErrorNotReady) return e;
            if ((k & 63) == 63 &&
                std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() > spin_ns)
                break;
        }
    }
    return hipEventSynchronize(ev);
}

__global__ void readback_kernel(const Readback r) {
    for (int i = 0; i < r.count; ++i)
        for (int j = threadIdx.x; j < r.n[i]; j += blockDim.x)
            __hip_atomic_store(r.dst[i] + j, r.src[i][j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (r.clamp_dst)
        for (int j = threadIdx.x; j < r.clamp_n; j += blockDim.x) {
            const int v = r.clamp_src[j];
            r.clamp_dst[j] = v >= 2 && v <= r.clamp_max ? v : 0;
        }
    if (r.seq_dst) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's stores have landed
        __syncthreads();
        if (threadIdx.x == 0) release_word_system(r.seq_dst, r.seq);
    }
}

hipError_t spin_word(const int* p, int want, hipStream_t s) {
    static const long long spin_ns = [] {
        const char* v = std::getenv("TTS_SPIN_MS");
        return (long long)((v && v[0]) ? std::atof(v) * 1e6 : 200e6);
    }();
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned k = 0;; ++k) {
        if (__atomic_load_n(p, __ATOMIC_ACQUIRE) == want) return hipSuccess;
        if ((k & 63) == 63 &&
            std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() > spin_ns)
            break;
    }
    hipError_t e = hipStreamSynchronize(s);  // a long run (or a fault): block, then look again
    if (e != hipSuccess) return e;
    return __atomic_load_n(p, __ATOMIC_ACQUIRE) == want ? hipSuccess : hipErrorUnknown;
}

hipError_t readback(const Readback& r, hipStream_t s) {
    if (r.count < 0 || r.count > 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(readback_kernel, dim3(1), dim3(64), 0, s, r);
    return hipGetLastError();
}

__global__ void stage_ids_kernel(const StageIds a) {
    for (int i = threadIdx.x; i < a.n; i += blockDim.x) a.ids[i] = a.v[i];
    if (threadIdx.x == 0) a.lens[0] = a.len;
}

hipError_t stage_ids(const StageIds& a, hipStream_t s) {
    if (a.n < 1 || a.n > STAGE_IDS_MAX) return hipErrorInvalidValue;
    hipLaunchKernelGGL(stage_ids_kernel, dim3(1), dim3(256), 0, s, a);
    return hipGetLastError();
}

__global__ void frag_mirror_kernel(const float* src, int64_t ld, int B, int K, float* dst, int ntf) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * K) return;
    const int b = i / K, k = i % K;
    dst[frag_idx(b, k, ntf)] = src[(int64_t)b * ld + k];
}

hipError_t frag_mirror(const float* src, int64_t ld, int B, int K, float* dst, int ntf, hipStream_t s) {
    const int n = B * K;
    hipLaunchKernelGGL(frag_mirror_kernel, dim3((n + 255) / 256), dim3(256), 0, s, src, ld, B, K, dst, ntf);
    return hipGetLastError();
}

}  // namespace tts

extern "C" {
const char* tts_last_error(void) { return tts::g_last_error.c_str(); }
const char* tts_version(void) { return "libtts_hip 0.1 (gfx950)"; }
}
