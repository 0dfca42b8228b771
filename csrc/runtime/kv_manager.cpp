// Native KV-cache block manager with prefix caching, plus the per-step batch
// metadata builder (positions / slot mapping / block tables / seq lens).
//
// This is the runtime counterpart of vLLM's block manager that the reference
// configures with --block-size 128 and --max-num-seqs 288
// (core/helm-charts/vllm/gaudi-values.yaml:160).  It lives in C++ because it
// runs on every engine step for every running sequence.
//
// Invariants (checked by check_invariants(), exercised by tests):
//   * ref[b] == number of live sequences whose table holds b
//   * a block is in the free list  <=>  ref[b] == 0
//   * a cached hash maps to a block whose stored hash equals it
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <cstring>
#include <list>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

inline uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

// Chained block hash: depends on the parent block's hash and this block's tokens.
inline uint64_t block_hash(uint64_t parent, const int32_t* toks, int n, uint64_t salt) {
  uint64_t h = mix64(parent ^ 0x9E3779B97F4A7C15ULL ^ salt);
  for (int i = 0; i < n; ++i) h = mix64(h ^ (uint64_t)(uint32_t)toks[i] * 0x100000001B3ULL + i);
  return h == 0 ? 1 : h;
}

struct SeqState {
  std::vector<int32_t> blocks;
  int num_hashed_blocks = 0;   // full blocks whose hash is registered
  uint64_t last_hash = 0;
};

class KVCacheManager {
 public:
  KVCacheManager(int num_blocks, int block_size, bool prefix_caching)
      : num_blocks_(num_blocks), block_size_(block_size), prefix_caching_(prefix_caching),
        ref_(num_blocks, 0), hash_(num_blocks, 0), pos_(num_blocks) {
    if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("bad kv geometry");
    for (int b = 0; b < num_blocks; ++b) pos_[b] = free_.insert(free_.end(), b);
  }

  int num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  int num_free_blocks() const { return (int)free_.size(); }
  double usage() const { return 1.0 - (double)free_.size() / (double)num_blocks_; }
  bool has_seq(int64_t sid) const { return seqs_.count(sid) != 0; }
  int num_seq_blocks(int64_t sid) const {
    auto it = seqs_.find(sid);
    return it == seqs_.end() ? 0 : (int)it->second.blocks.size();
  }

  // Look up the longest cached full-block prefix of `tokens` and attach those
  // blocks to a NEW sequence. Returns the number of cached tokens. Never returns
  // the whole prompt: at least one token must be recomputed to produce logits.
  int allocate_prefix(int64_t sid, py::array_t<int32_t, py::array::c_style> tokens, uint64_t salt) {
    if (seqs_.count(sid)) throw std::runtime_error("sequence already allocated");
    SeqState st;
    const int n = (int)tokens.size();
    const int32_t* t = tokens.data();
    int cached_tokens = 0;
    if (prefix_caching_) {
      uint64_t h = 0;
      const int max_full = (n - 1) / block_size_;
      for (int i = 0; i < max_full; ++i) {
        h = block_hash(h, t + i * block_size_, block_size_, salt);
        auto it = cached_.find(h);
        if (it == cached_.end()) break;
        const int b = it->second;
        if (ref_[b] == 0) free_.erase(pos_[b]);
        ++ref_[b];
        st.blocks.push_back(b);
        st.num_hashed_blocks = i + 1;
        st.last_hash = h;
        cached_tokens += block_size_;
        ++hits_;
      }
      queries_ += max_full;
    }
    seqs_.emplace(sid, std::move(st));
    return cached_tokens;
  }

  // Blocks needed to grow `sid` to hold `num_tokens` tokens.
  int blocks_needed(int64_t sid, int num_tokens) const {
    auto it = seqs_.find(sid);
    const int have = it == seqs_.end() ? 0 : (int)it->second.blocks.size();
    const int need = (num_tokens + block_size_ - 1) / block_size_;
    return need > have ? need - have : 0;
  }

  // Grow the table; returns false (and allocates nothing) if not enough blocks.
  bool ensure(int64_t sid, int num_tokens) {
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) it = seqs_.emplace(sid, SeqState{}).first;
    const int extra = blocks_needed(sid, num_tokens);
    if (extra > (int)free_.size()) return false;
    for (int i = 0; i < extra; ++i) it->second.blocks.push_back(pop_free());
    return true;
  }

  // Register hashes of newly completed full blocks (prefix caching).
  void commit(int64_t sid, py::array_t<int32_t, py::array::c_style> tokens, int num_computed,
              uint64_t salt) {
    if (!prefix_caching_) return;
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) return;
    SeqState& st = it->second;
    const int32_t* t = tokens.data();
    const int nfull = std::min<int>(num_computed, (int)tokens.size()) / block_size_;
    for (int i = st.num_hashed_blocks; i < nfull && i < (int)st.blocks.size(); ++i) {
      const uint64_t h = block_hash(st.last_hash, t + i * block_size_, block_size_, salt);
      const int b = st.blocks[i];
      if (hash_[b] == 0) {
        auto c = cached_.find(h);
        if (c == cached_.end()) {
          cached_.emplace(h, b);
          hash_[b] = h;
        }
      }
      st.last_hash = h;
      st.num_hashed_blocks = i + 1;
    }
  }

  void free_seq(int64_t sid) {
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) return;
    auto& blocks = it->second.blocks;
    // release tail first so the LRU evicts the least shareable blocks first
    for (int i = (int)blocks.size() - 1; i >= 0; --i) {
      const int b = blocks[i];
      if (--ref_[b] == 0) pos_[b] = free_.insert(free_.end(), b);
    }
    seqs_.erase(it);
  }

  // Share the blocks of `src` with a new sequence `dst` (n > 1 sampling / beam).
  void fork(int64_t src, int64_t dst) {
    auto it = seqs_.find(src);
    if (it == seqs_.end()) throw std::runtime_error("fork: unknown source");
    SeqState st = it->second;
    for (int b : st.blocks) ++ref_[b];
    seqs_[dst] = st;
  }

  // Copy-on-write for the last block of `sid` if it is shared; returns
  // (src_block, dst_block) or (-1, -1) when no copy is needed.
  std::pair<int, int> cow_last(int64_t sid) {
    auto it = seqs_.find(sid);
    if (it == seqs_.end() || it->second.blocks.empty()) return {-1, -1};
    int& last = it->second.blocks.back();
    if (ref_[last] <= 1) return {-1, -1};
    if (free_.empty()) throw std::runtime_error("cow: out of blocks");
    const int nb = pop_free();
    --ref_[last];
    const int old = last;
    last = nb;
    return {old, nb};
  }

  std::vector<int32_t> block_table(int64_t sid) const {
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) return {};
    return it->second.blocks;
  }

  void reset_prefix_cache() {
    for (auto& kv : cached_) hash_[kv.second] = 0;
    cached_.clear();
  }

  // ---- per-step metadata builder ------------------------------------------------
  // For entry i: sequence seq_ids[i] computes tokens [starts[i], starts[i]+counts[i]).
  // Writes (flattened over entries):
  //   positions[T], slots[T]
  //   block_tables[n, bt_stride] (row i; zero padded), seq_lens[n] = starts+counts
  // Returns T.
  int build(py::array_t<int64_t, py::array::c_style> seq_ids,
            py::array_t<int32_t, py::array::c_style> starts,
            py::array_t<int32_t, py::array::c_style> counts,
            uintptr_t positions_ptr, uintptr_t slots_ptr, uintptr_t block_tables_ptr,
            int bt_stride, uintptr_t seq_lens_ptr, int max_tokens) const {
    const int n = (int)seq_ids.size();
    int32_t* positions = reinterpret_cast<int32_t*>(positions_ptr);
    int32_t* slots = reinterpret_cast<int32_t*>(slots_ptr);
    int32_t* bts = reinterpret_cast<int32_t*>(block_tables_ptr);
    int32_t* lens = reinterpret_cast<int32_t*>(seq_lens_ptr);
    const int64_t* ids = seq_ids.data();
    const int32_t* st = starts.data();
    const int32_t* ct = counts.data();
    int T = 0;
    for (int i = 0; i < n; ++i) {
      auto it = seqs_.find(ids[i]);
      if (it == seqs_.end()) throw std::runtime_error("build: unknown sequence");
      const auto& blocks = it->second.blocks;
      const int end = st[i] + ct[i];
      if ((end + block_size_ - 1) / block_size_ > (int)blocks.size())
        throw std::runtime_error("build: sequence table too short");
      if ((int)blocks.size() > bt_stride) throw std::runtime_error("build: bt_stride too small");
      if (T + ct[i] > max_tokens) throw std::runtime_error("build: token buffer overflow");
      for (int p = st[i]; p < end; ++p) {
        positions[T] = p;
        slots[T] = blocks[p / block_size_] * block_size_ + (p % block_size_);
        ++T;
      }
      if (bts) {
        int32_t* row = bts + (int64_t)i * bt_stride;
        const int nb = (int)blocks.size();
        std::memcpy(row, blocks.data(), sizeof(int32_t) * nb);
        std::memset(row + nb, 0, sizeof(int32_t) * (bt_stride - nb));
      }
      if (lens) lens[i] = end;
    }
    return T;
  }

  std::string check_invariants() const {
    std::vector<int> cnt(num_blocks_, 0);
    for (auto& kv : seqs_)
      for (int b : kv.second.blocks) {
        if (b < 0 || b >= num_blocks_) return "block id out of range";
        ++cnt[b];
      }
    std::vector<char> in_free(num_blocks_, 0);
    for (int b : free_) {
      if (in_free[b]) return "block twice in free list";
      in_free[b] = 1;
    }
    for (int b = 0; b < num_blocks_; ++b) {
      if (cnt[b] != ref_[b]) return "refcount mismatch at block " + std::to_string(b);
      if ((ref_[b] == 0) != (bool)in_free[b]) return "free-list mismatch at block " + std::to_string(b);
    }
    for (auto& kv : cached_)
      if (hash_[kv.second] != kv.first) return "stale cache entry";
    return "";
  }

  py::dict stats() const {
    py::dict d;
    d["num_blocks"] = num_blocks_;
    d["free_blocks"] = (int)free_.size();
    d["cached_blocks"] = (int)cached_.size();
    d["prefix_hits"] = hits_;
    d["prefix_queries"] = queries_;
    d["num_seqs"] = (int)seqs_.size();
    return d;
  }

 private:
  int pop_free() {
    const int b = free_.front();
    free_.pop_front();
    if (hash_[b] != 0) {       // evict cached content
      auto c = cached_.find(hash_[b]);
      if (c != cached_.end() && c->second == b) cached_.erase(c);
      hash_[b] = 0;
    }
    ref_[b] = 1;
    return b;
  }

  int num_blocks_, block_size_;
  bool prefix_caching_;
  std::vector<int> ref_;
  std::vector<uint64_t> hash_;
  std::list<int> free_;
  std::vector<std::list<int>::iterator> pos_;
  std::unordered_map<uint64_t, int> cached_;
  std::unordered_map<int64_t, SeqState> seqs_;
  int64_t hits_ = 0, queries_ = 0;
};

}  // namespace

void register_shm(py::module_& m);       // shm_ring.cpp
void register_grammar(py::module_& m);   // grammar.cpp

PYBIND11_MODULE(_eia_runtime, m) {
  m.doc() = "MI355X inference runtime: native KV block manager, batch builder, shm broadcast";
  py::class_<KVCacheManager>(m, "KVCacheManager")
      .def(py::init<int, int, bool>(), py::arg("num_blocks"), py::arg("block_size"),
           py::arg("prefix_caching") = true)
      .def_property_readonly("num_blocks", &KVCacheManager::num_blocks)
      .def_property_readonly("block_size", &KVCacheManager::block_size)
      .def("num_free_blocks", &KVCacheManager::num_free_blocks)
      .def("usage", &KVCacheManager::usage)
      .def("has_seq", &KVCacheManager::has_seq)
      .def("num_seq_blocks", &KVCacheManager::num_seq_blocks)
      .def("allocate_prefix", &KVCacheManager::allocate_prefix, py::arg("seq_id"),
           py::arg("tokens"), py::arg("salt") = 0)
      .def("blocks_needed", &KVCacheManager::blocks_needed)
      .def("ensure", &KVCacheManager::ensure)
      .def("commit", &KVCacheManager::commit, py::arg("seq_id"), py::arg("tokens"),
           py::arg("num_computed"), py::arg("salt") = 0)
      .def("free", &KVCacheManager::free_seq)
      .def("fork", &KVCacheManager::fork)
      .def("cow_last", &KVCacheManager::cow_last)
      .def("block_table", &KVCacheManager::block_table)
      .def("reset_prefix_cache", &KVCacheManager::reset_prefix_cache)
      .def("build", &KVCacheManager::build)
      .def("check_invariants", &KVCacheManager::check_invariants)
      .def("stats", &KVCacheManager::stats);
  register_shm(m);
  register_grammar(m);
}
