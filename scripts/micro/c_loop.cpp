// Micro harness: K back-to-back drcvar_safe_halfspaces_f64 calls issued from native code (what a
// C/C++ control loop calling the ABI does), to time against hipGraph replays (c_loop.py).
#include <cstdint>
#include "drcvar_halfspace.h"
extern "C" int c_loop(int k, const double* s, int64_t o, int64_t t, int64_t n, int64_t so,
                      int64_t st, int64_t sn, const double* ego, int64_t es, double rr, double ro,
                      double alpha, double delta, double eps, double* out, void* stream) {
  for (int i = 0; i < k; ++i) {
    const int c = drcvar_safe_halfspaces_f64(s, o, t, n, so, st, sn, ego, es, rr, ro, alpha, delta,
                                             eps, out, stream);
    if (c) return c;
  }
  return 0;
}
