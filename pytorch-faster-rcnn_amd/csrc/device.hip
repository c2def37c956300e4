// Per-device properties the launch planning needs (common.h resident_capacity).
#include <mutex>
#include <utility>
#include <vector>

#include "common.h"

namespace frh {

int resident_capacity(const void* kernel, int block, size_t dyn_lds) {
  // (device, kernel, block, dyn_lds) -> capacity; a handful of entries per process
  struct Ent {
    int dev;
    const void* k;
    int block;
    size_t lds;
    int cap;
  };
  static std::mutex mu;
  static std::vector<Ent> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  {
    std::lock_guard<std::mutex> g(mu);
    for (const Ent& e : cache)
      if (e.dev == dev && e.k == kernel && e.block == block && e.lds == dyn_lds) return e.cap;
  }
  int ncu = 0, per_cu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, dyn_lds) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  const int cap = ncu * per_cu;
  std::lock_guard<std::mutex> g(mu);
  cache.push_back(Ent{dev, kernel, block, dyn_lds, cap});
  return cap;
}

}  // namespace frh
