// Paged KV-cache block manager for one pipeline shard (header-only core; the pybind11 module is
// block_manager.cpp, the sanitizer stress test test_block_manager.cpp).
//
// The reference keeps ONE global KV cache per engine, sized prompt_len + 1024 and reset on every
// prompt (xotorch/inference/torch/sharded_inference_engine.py:71-82,134-147), so concurrent requests
// clobber each other.  Here every request owns a list of 64-token pages in a shard-wide pool sized
// for the GPU's HBM (288 GB on MI355X); the scheduler asks this manager for the cache slots of the
// tokens it is about to run and for dense block tables / context lengths of a batch, written
// straight into caller-owned (pinned) int32 buffers that are then copied to the device.
// Not internally synchronised: each engine drives it from its single executor thread.
#pragma once
#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace xot_rt {

class BlockManager {
 public:
  BlockManager(int64_t num_blocks, int64_t block_size) : block_size_(block_size), refcnt_(num_blocks, 0) {
    if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("num_blocks and block_size must be > 0");
    free_.reserve(num_blocks);
    for (int64_t b = num_blocks - 1; b >= 0; --b) free_.push_back((int32_t)b);  // pop_back hands out 0,1,2,...
  }

  int64_t block_size() const { return block_size_; }
  int64_t num_blocks() const { return (int64_t)refcnt_.size(); }
  int64_t num_free() const { return (int64_t)free_.size(); }
  bool has(const std::string& rid) const { return seqs_.count(rid) != 0; }
  int64_t num_tokens(const std::string& rid) const { return get(rid).ntok; }
  int64_t num_sequences() const { return (int64_t)seqs_.size(); }

  int64_t blocks_needed(const std::string& rid, int64_t extra_tokens) const {
    auto it = seqs_.find(rid);
    const int64_t have_tok = it == seqs_.end() ? 0 : it->second.ntok;
    const int64_t have_blk = it == seqs_.end() ? 0 : (int64_t)it->second.blocks.size();
    const int64_t need_blk = (have_tok + extra_tokens + block_size_ - 1) / block_size_;
    return std::max<int64_t>(0, need_blk - have_blk);
  }
  bool can_append(const std::string& rid, int64_t extra_tokens) const {
    return blocks_needed(rid, extra_tokens) <= num_free();
  }

  // Reserve cache slots for `n` new tokens of request `rid`; returns their global slot ids
  // (block * block_size + offset) in order.  Throws (allocating nothing) when the pool is exhausted.
  std::vector<int64_t> append(const std::string& rid, int64_t n) {
    if (n < 0) throw std::invalid_argument("append: n < 0");
    const int64_t need = blocks_needed(rid, n);
    if (need > num_free()) throw std::runtime_error("KV cache exhausted: need " + std::to_string(need) + " pages, " + std::to_string(num_free()) + " free");
    Seq& s = seqs_[rid];
    for (int64_t i = 0; i < need; ++i) {
      const int32_t b = free_.back();
      free_.pop_back();
      refcnt_[b] = 1;
      s.blocks.push_back(b);
    }
    std::vector<int64_t> slots(n);
    for (int64_t i = 0; i < n; ++i) {
      const int64_t t = s.ntok + i;
      slots[i] = (int64_t)s.blocks[t / block_size_] * block_size_ + t % block_size_;
    }
    s.ntok += n;
    return slots;
  }

  // Drop the last n tokens (e.g. a speculative or aborted step); frees pages that become empty.
  void truncate(const std::string& rid, int64_t new_len) {
    Seq& s = getm(rid);
    if (new_len < 0 || new_len > s.ntok) throw std::invalid_argument("truncate: bad length");
    s.ntok = new_len;
    const size_t keep = (size_t)((new_len + block_size_ - 1) / block_size_);
    while (s.blocks.size() > keep) {
      release(s.blocks.back());
      s.blocks.pop_back();
    }
  }

  void free_seq(const std::string& rid) {
    auto it = seqs_.find(rid);
    if (it == seqs_.end()) return;
    for (int32_t b : it->second.blocks) release(b);
    seqs_.erase(it);
  }

  // Share the first `ntok` tokens' full pages of `src` with a new request `dst` (prefix reuse).
  void fork(const std::string& src, const std::string& dst, int64_t ntok) {
    const Seq& s = get(src);
    if (seqs_.count(dst)) throw std::invalid_argument("fork: destination exists");
    ntok = std::min<int64_t>(ntok, s.ntok) / block_size_ * block_size_;  // whole pages only
    Seq d;
    for (int64_t i = 0; i < ntok / block_size_; ++i) {
      d.blocks.push_back(s.blocks[i]);
      refcnt_[s.blocks[i]] += 1;
    }
    d.ntok = ntok;
    seqs_[dst] = std::move(d);
  }

  std::vector<int32_t> block_table(const std::string& rid) const { return get(rid).blocks; }

  // Fill a dense [B, width] int32 block table and [B] context lengths for a batch.  Rows shorter
  // than `width` are padded with block 0 (never read: the kernels stop at the context length).
  void fill_batch(const std::vector<std::string>& rids, int32_t* tables, int64_t rows, int64_t width,
                  int32_t* ctx_lens, int64_t ctx_rows) const {
    if ((int64_t)rids.size() > rows || (int64_t)rids.size() > ctx_rows)
      throw std::invalid_argument("fill_batch: buffers too small");
    for (size_t i = 0; i < rids.size(); ++i) {
      const Seq& s = get(rids[i]);
      if ((int64_t)s.blocks.size() > width) throw std::invalid_argument("fill_batch: block table too narrow");
      int32_t* row = tables + (int64_t)i * width;
      for (int64_t j = 0; j < width; ++j) row[j] = j < (int64_t)s.blocks.size() ? s.blocks[j] : 0;
      ctx_lens[i] = (int32_t)s.ntok;
    }
  }

  // Consistency check (tests / sanitizer runs): every page is either free exactly once or referenced
  // by the sequences that hold it, with matching reference counts.
  bool check() const {
    std::vector<int32_t> refs(refcnt_.size(), 0);
    for (const auto& kv : seqs_) {
      if ((int64_t)kv.second.blocks.size() != (kv.second.ntok + block_size_ - 1) / block_size_) return false;
      for (int32_t b : kv.second.blocks) {
        if (b < 0 || b >= (int32_t)refcnt_.size()) return false;
        refs[b]++;
      }
    }
    std::vector<char> freed(refcnt_.size(), 0);
    for (int32_t b : free_) {
      if (b < 0 || b >= (int32_t)refcnt_.size() || freed[b] || refs[b] != 0) return false;
      freed[b] = 1;
    }
    for (size_t b = 0; b < refcnt_.size(); ++b)
      if (refs[b] != refcnt_[b] || (refs[b] == 0) != (freed[b] != 0)) return false;
    return true;
  }

 private:
  struct Seq {
    std::vector<int32_t> blocks;
    int64_t ntok = 0;
  };
  const Seq& get(const std::string& rid) const {
    auto it = seqs_.find(rid);
    if (it == seqs_.end()) throw std::out_of_range("unknown request " + rid);
    return it->second;
  }
  Seq& getm(const std::string& rid) {
    auto it = seqs_.find(rid);
    if (it == seqs_.end()) throw std::out_of_range("unknown request " + rid);
    return it->second;
  }
  void release(int32_t b) {
    if (--refcnt_[b] == 0) free_.push_back(b);
  }

  int64_t block_size_;
  std::vector<int32_t> refcnt_;
  std::vector<int32_t> free_;
  std::unordered_map<std::string, Seq> seqs_;
};

}  // namespace xot_rt
