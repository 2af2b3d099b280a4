// Host-side sanitizer run of the native .dat reader (ASan on the CPU-side native code).
// Usage: dat_reader_asan <file>...  — prints "<rows> <cols> <rc> <sum>" per file; malformed files must
// come back as SYSID_E_INVALID without any out-of-bounds access.
#include <cstdint>
#include <cstdio>
#include <vector>

#include "sysid.h"

int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i) {
    int64_t r = 0, c = 0;
    int rc = sysid_dat_shape(argv[i], &r, &c);
    double sum = 0.0;
    if (rc == SYSID_OK) {
      std::vector<float> buf((size_t)(r * c) + 1);
      for (int t : {1, 3, 8}) {
        rc = sysid_dat_read(argv[i], buf.data(), r, c, t);
        if (rc != SYSID_OK) break;
      }
      for (int64_t k = 0; k < r * c && rc == SYSID_OK; ++k) sum += buf[(size_t)k];
    }
    std::printf("%lld %lld %d %.9g\n", (long long)r, (long long)c, rc, sum);
  }
  return 0;
}
