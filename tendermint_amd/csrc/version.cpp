// tmv_version(): the library's version with the build id the Makefile
// generates ($(OUT)/build_id.h: digest of the sources, git HEAD).
#include "build_id.h"

extern "C" const char *tmv_version(void) {
  return "tmverify-mi355x 0.4 (gfx950) src=" TMV_SRC_DIGEST " git=" TMV_GIT_HEAD;
}
