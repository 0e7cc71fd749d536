// Randomised stress test of the block manager, built with host AddressSanitizer + UBSan by
// tests/test_native_sanitizers.py (GPU sanitizers are not available; the host runtime is checked
// here).  Exit code 0 = every invariant held.
#include <cstdio>
#include <random>

#include "block_manager.h"

int main() {
  std::mt19937 rng(12345);
  for (int trial = 0; trial < 20; ++trial) {
    const int64_t nblocks = 16 + rng() % 200, bs = (rng() % 2) ? 64 : 16;
    xot_rt::BlockManager bm(nblocks, bs);
    std::vector<std::string> live;
    for (int op = 0; op < 4000; ++op) {
      const int kind = rng() % 6;
      if (kind <= 1 || live.empty()) {  // new request (prefill)
        const std::string rid = "r" + std::to_string(trial) + "_" + std::to_string(op);
        const int64_t n = 1 + rng() % (3 * bs);
        if (bm.can_append(rid, n)) {
          auto slots = bm.append(rid, n);
          if ((int64_t)slots.size() != n) return 1;
          live.push_back(rid);
        } else {
          try {
            bm.append(rid, n);
            return 2;  // must throw
          } catch (const std::runtime_error&) {
          }
          if (bm.has(rid) && bm.num_tokens(rid) != 0) return 3;
          bm.free_seq(rid);
        }
      } else if (kind == 2) {  // decode step
        const std::string& rid = live[rng() % live.size()];
        if (bm.can_append(rid, 1)) bm.append(rid, 1);
      } else if (kind == 3) {  // finish
        const size_t i = rng() % live.size();
        bm.free_seq(live[i]);
        live.erase(live.begin() + i);
      } else if (kind == 4) {  // truncate
        const std::string& rid = live[rng() % live.size()];
        bm.truncate(rid, bm.num_tokens(rid) / 2);
      } else {  // prefix fork
        const std::string& src = live[rng() % live.size()];
        const std::string dst = src + "_f" + std::to_string(op);
        bm.fork(src, dst, bm.num_tokens(src));
        live.push_back(dst);
      }
      if (!bm.check()) {
        std::printf("invariant broken: trial %d op %d\n", trial, op);
        return 4;
      }
    }
    // batch tables for whatever is live
    const int64_t width = nblocks;
    std::vector<int32_t> tables(live.size() * width), ctx(live.size());
    bm.fill_batch(live, tables.data(), (int64_t)live.size(), width, ctx.data(), (int64_t)live.size());
    for (size_t i = 0; i < live.size(); ++i)
      if (ctx[i] != bm.num_tokens(live[i])) return 5;
    for (const auto& r : live) bm.free_seq(r);
    if (bm.num_free() != nblocks || !bm.check()) return 6;
  }
  std::printf("block manager stress: ok\n");
  return 0;
}
