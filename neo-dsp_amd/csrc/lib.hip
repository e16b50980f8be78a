// lib.hip — library-wide C-ABI entry points (error latch, version, devices).
#include "common.hpp"

namespace neo_hip {
std::string& last_error_slot()
{
    thread_local std::string slot;
    return slot;
}
}  // namespace neo_hip

extern "C" {

NEO_HIP_API const char* neo_hip_last_error(void) { return neo_hip::last_error_slot().c_str(); }

NEO_HIP_API int neo_hip_version(void) { return NEO_HIP_VERSION; }

NEO_HIP_API int neo_hip_device_count(int* count)
{
    if (!count) return neo_hip::fail(NEO_HIP_EINVAL, "count is null");
    *count = 0;
    hipError_t e = hipGetDeviceCount(count);
    if (e != hipSuccess) {
        *count = 0;
        return neo_hip::fail(NEO_HIP_ENODEV, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_host_register(void* p, int64_t bytes)
{
    if (!p || bytes <= 0) return neo_hip::fail(NEO_HIP_EINVAL, "null pointer or empty range");
    NEO_HIP_CHECK(hipHostRegister(p, size_t(bytes), hipHostRegisterMapped | hipHostRegisterPortable));
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_host_unregister(void* p)
{
    if (!p) return neo_hip::fail(NEO_HIP_EINVAL, "null pointer");
    NEO_HIP_CHECK(hipHostUnregister(p));
    return NEO_HIP_OK;
}

}  // extern "C"
