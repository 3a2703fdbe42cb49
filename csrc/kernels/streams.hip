// Stream-ordering edges for the engines' side branches without Python stream objects: stream_fork(src, dst) makes
// dst wait for everything enqueued on src so far (hipEventRecord + hipStreamWaitEvent on a pooled event).  A wait
// binds to the event's latest record at the time of the call, so the pool's events are reused round-robin.  The
// ResNet-18-GN engine forks its weight-gradient branch ~45 times per step; torch.cuda.Stream.wait_stream plus a
// `with torch.cuda.stream(...)` block cost ~30 us of host time per fork, which left the GPU idle 6-7 % of a CIFAR
// SubAvg round (profiles/r5_subavg_round_kernels_branch.txt).
#include <map>
#include <utility>
#include <vector>

#include "common.h"

namespace nidt {

// One pool per device: an event recorded on a stream must belong to that stream's device.
void stream_fork(uintptr_t src, uintptr_t dst) {
  static std::map<int, std::pair<std::vector<hipEvent_t>, size_t>> pools;
  int dev = 0;
  NIDT_CHECK(hipGetDevice(&dev));
  auto& pl = pools[dev];
  auto& pool = pl.first;
  if (pool.empty()) {
    pool.resize(64);
    for (auto& e : pool) NIDT_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  hipEvent_t e = pool[pl.second++ % pool.size()];
  NIDT_CHECK(hipEventRecord(e, as_stream(src)));
  NIDT_CHECK(hipStreamWaitEvent(as_stream(dst), e, 0));
}

}  // namespace nidt
