// Live kernel timing (profiling aid for bench.py's roofline object): while
// on, the launches of a few hot kernels are bracketed by timing events on the
// stream they are launched on; read() resolves the finished pairs into a
// total duration and a launch count.  Off by default (two event records per
// timed launch when on).  Implemented in msm_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tmv {
namespace ktimer {

enum Kernel : int { kAccum = 0, kWpart = 1, kPrep = 2, kCount = 3 };

void set(bool on);
bool on();
// begin() returns a token (nullptr when off); end() records the closing event.
void *begin(Kernel k, hipStream_t s);
void end(void *token, hipStream_t s);
// Waits for the recorded pairs of kernel k, adds them to *ms / *launches and
// forgets them.  0 or a HIP error.
int read(Kernel k, double *ms, uint64_t *launches);

}  // namespace ktimer
}  // namespace tmv
