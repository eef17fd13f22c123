// capi.cpp — library-level C-ABI entry points: version, last error, device binding.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>

#include "common.hpp"

namespace mage {

namespace {
thread_local std::string g_last_error;
}

void set_error(const std::string& msg) { g_last_error = msg; }
const char* last_error() { return g_last_error.c_str(); }

mage_status bind_device(int device)
{
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
        set_error("no HIP device available");
        return MAGE_EDEVICE;
    }
    if (device < 0 || device >= count) {
        set_error("device index " + std::to_string(device) + " out of range");
        return MAGE_EDEVICE;
    }
    MAGE_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    MAGE_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_error(std::string("device is ") + prop.gcnArchName + ", this build targets gfx950 only");
        return MAGE_EDEVICE;
    }
    return MAGE_OK;
}

}  // namespace mage

extern "C" {

const char* mage_version(void) { return "mageslam_amd 0.1.0 (gfx950)"; }
const char* mage_last_error(void) { return mage::last_error(); }

}
