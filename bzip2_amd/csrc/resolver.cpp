// resolver.cpp -- see resolver.h.
#include "resolver.h"

#include <hip/hip_runtime.h>

#include <map>
#include <string>

namespace bzg {

int32_t periodic_origptr(const uint8_t* blk, int32_t n) {
  (void)blk;
  (void)n;
  throw ResolverFailure();  // A5 tie order not implemented yet
}

void resolve_origptrs(const uint8_t* d_blk, const std::vector<uint32_t>& boff, const std::vector<uint32_t>& period,
                      std::vector<uint32_t>& rank) {
  const size_t nb = rank.size();
  std::map<std::string, int32_t> memo;  // identical periodic blocks resolve once
  for (size_t b = 0; b < nb; b++) {
    const uint32_t n = boff[b + 1] - boff[b], p = period[b];
    const uint32_t k = n / p;
    if (k == 1) continue;                // aperiodic: the rank is the origPtr
    if (p == 1) { rank[b] = 0; continue; }  // one symbol: no B* suffix, origPtr 0 (blocksort.c:1349)
    std::string bytes(n, '\0');
    if (hipMemcpy(&bytes[0], d_blk + boff[b], n, hipMemcpyDeviceToHost) != hipSuccess) throw ResolverFailure();
    auto it = memo.find(bytes);
    if (it == memo.end()) it = memo.emplace(bytes, periodic_origptr((const uint8_t*)bytes.data(), (int32_t)n)).first;
    rank[b] = (uint32_t)it->second;
  }
}

}  // namespace bzg
