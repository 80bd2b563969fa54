// Error reporting shared by every entry point of libtts_hip.
#include <cstdio>
#include <cstdlib>
#include <string>

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

hipError_t launch_persistent(const void* fn, dim3 grid, dim3 block, void** args, size_t smem, hipStream_t s,
                             bool* launched) {
    *launched = false;
    const long long blocks = (long long)grid.x * grid.y * grid.z;
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, (int)(block.x * block.y * block.z), smem);
    if (e != hipSuccess) return e;
    if ((long long)per_cu * usable_cus() < blocks) return hipSuccess;  // cannot be co-resident: fall back
    const char* coop = std::getenv("TTS_COOP");
    if (coop && coop[0] == '0') {
        e = hipLaunchKernel(fn, grid, block, args, smem, s);
    } else {
        e = hipLaunchCooperativeKernel(fn, grid, block, args, (unsigned)smem, s);
        if (e == hipErrorCooperativeLaunchTooLarge) {
            (void)hipGetLastError();  // refused before anything ran: fall back
            return hipSuccess;
        }
    }
    if (e == hipSuccess) *launched = true;
    return e;
}

}  // namespace tts

extern "C" {
const char* tts_last_error(void) { return tts::g_last_error.c_str(); }
const char* tts_version(void) { return "libtts_hip 0.1 (gfx950)"; }
}
