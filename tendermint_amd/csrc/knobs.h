// Environment knobs of libtmgpu.so.
//
// Production knobs (INTEGRATION.md lists them) are thresholds, sizes,
// timeouts and capacities, each read with getenv where it is used.  A/B
// switches -- alternatives measured during development, kept so that a
// same-box A/B can be re-run -- are read through ab_knob(), which only a
// build made with -DTMV_AB (tools/build_ab.sh) compiles in: the product
// library ignores them, so no deployment environment can steer its verdict
// path onto a variant.
#pragma once
#include <cstdlib>

namespace tmv {

inline const char *ab_knob(const char *name) {
#ifdef TMV_AB
  return std::getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

}  // namespace tmv
