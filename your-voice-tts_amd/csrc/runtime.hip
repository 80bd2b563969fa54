// Error reporting shared by every entry point of libtts_hip.
#include <cstdio>
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

}  // namespace tts

extern "C" {
const char* tts_last_error(void) { return tts::g_last_error.c_str(); }
const char* tts_version(void) { return "libtts_hip 0.1 (gfx950)"; }
}
