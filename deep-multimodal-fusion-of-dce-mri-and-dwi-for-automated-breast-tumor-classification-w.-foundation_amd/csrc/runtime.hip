// Library-wide state of the C-ABI: error buffer, version, RNG state helpers.
#include "dmf_common.h"
#include "../../include/dmf_hip.h"
#include <string.h>

namespace dmf {
static thread_local char g_err[1024] = {0};
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace dmf

extern "C" const char* dmf_last_error(void) { return dmf::g_err; }
extern "C" int dmf_abi_version(void) { return DMF_ABI_VERSION; }

// Probe kernel: y[i] = a * i + b. Used by the smoke path to check that the
// code object loads on the device and that torch's stream handle is honoured.
__global__ void k_iota(float* y, long long n, float a, float b) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = a * (float)i + b;
}
extern "C" int dmf_iota_f32(float* y, long long n, float a, float b, void* stream) {
  DMF_CHECK_ARG(y != nullptr && n >= 0, "dmf_iota_f32: bad args (n=%lld)", n);
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_iota, dim3(dmf::cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, y, n, a, b);
  DMF_LAUNCH_CHECK("dmf_iota_f32");
  return 0;
}

// Advance a device-resident RNG offset (uint64 at p) by `inc` -- a graph-safe
// way to give each dropout site a fresh counter range on every replay.
__global__ void k_rng_advance(unsigned long long* p, unsigned long long inc) { *p += inc; }
extern "C" int dmf_rng_advance(unsigned long long* state, unsigned long long inc, void* stream) {
  DMF_CHECK_ARG(state != nullptr, "dmf_rng_advance: null state");
  hipLaunchKernelGGL(k_rng_advance, dim3(1), dim3(1), 0, (hipStream_t)stream, state, inc);
  DMF_LAUNCH_CHECK("dmf_rng_advance");
  return 0;
}
