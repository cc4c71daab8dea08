// Prints the HIP device attributes the launch code sizes itself by (CUs, LDS per CU / block).
// Build: hipcc --offload-arch=gfx950 -o .exp/devinfo tools/devinfo.hip
#include <hip/hip_runtime.h>

#include <cstdio>

int main() {
  const struct {
    hipDeviceAttribute_t a;
    const char* n;
  } at[] = {
      {hipDeviceAttributeMultiprocessorCount, "cus"},
      {hipDeviceAttributeMaxSharedMemoryPerBlock, "lds_per_block"},
      {hipDeviceAttributeSharedMemPerBlockOptin, "lds_per_block_optin"},
      {hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, "lds_per_cu"},
      {hipDeviceAttributeClockRate, "clock_khz"},
  };
  for (const auto& x : at) {
    int v = -1;
    (void)hipDeviceGetAttribute(&v, x.a, 0);
    printf("%s %d\n", x.n, v);
  }
  return 0;
}
