// Pushdown matcher for recursive ``guided_grammar`` constraints (engine/grammar.py).
//
// The reference serves guided decoding through vLLM's OpenAI surface (docs/api-spec.yaml
// guided_grammar); a grammar whose rules recurse is not a regular language, so the token FSM of
// engine/fsm.py cannot run it.  Here the grammar is a CFG over code-point classes and the
// matcher keeps the SET of parser stacks that are consistent with the text so far:
//
//   * a stack is an interned linked list of grammar positions (top = next symbol to match);
//     positions index one flat symbol array (class id >= 0, rule ref < 0, kEnd ends an
//     alternative).  After expansion every live stack's top is a class; the empty stack (-1)
//     means the start rule is complete.
//   * tail calls are eliminated (a return address that only ends its alternative is not
//     pushed), so ``X*`` / right recursion over a long string keeps the stacks shallow.
//   * stack cells and stack sets are interned per grammar, and (set, code point) -> set
//     transitions cached: the matcher is a lazily built automaton over stack sets, shared by
//     every request using the grammar (a string body loops on one state);
//   * mask(): one depth-first walk of the vocabulary trie from a state -- shared prefixes
//     stepped once, a branch dropped as soon as its set empties -- cached per state.
//
// Left recursion is rejected when the grammar is compiled (engine/grammar.py); the expansion
// additionally caps its depth so a hand-built grammar cannot loop.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <unordered_map>
#include <utility>
#include <vector>

namespace py = pybind11;

namespace {

constexpr int kEnd = INT_MIN;
constexpr size_t kMaxStacks = 4096;
constexpr int kMaxExpandDepth = 4096;
constexpr size_t kMaxMemo = 256;               // cached state masks per grammar

struct Grammar {
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> classes;
  std::vector<int> flat;                  // symbols of every alternative, kEnd-terminated
  std::vector<std::vector<int>> alts;     // rule -> start positions of its alternatives
  int start = 0;

  Grammar(std::vector<std::vector<std::pair<uint32_t, uint32_t>>> cls,
          const std::vector<std::vector<std::vector<int>>>& rules, int start_rule)
      : classes(std::move(cls)), start(start_rule) {
    const int nr = static_cast<int>(rules.size());
    if (start < 0 || start >= nr) throw std::invalid_argument("grammar: bad start rule");
    for (auto& c : classes) {                       // sorted, disjoint ranges
      std::sort(c.begin(), c.end());
      std::vector<std::pair<uint32_t, uint32_t>> m;
      for (const auto& r : c) {
        if (!m.empty() && r.first <= m.back().second + 1ull)
          m.back().second = std::max(m.back().second, r.second);
        else
          m.push_back(r);
      }
      c = std::move(m);
    }
    alts.resize(nr);
    for (int r = 0; r < nr; ++r) {
      for (const auto& a : rules[r]) {
        alts[r].push_back(static_cast<int>(flat.size()));
        for (int s : a) {
          if (s >= 0 && s >= static_cast<int>(classes.size()))
            throw std::invalid_argument("grammar: class id out of range");
          if (s < 0 && -s - 1 >= nr) throw std::invalid_argument("grammar: rule id out of range");
          flat.push_back(s);
        }
        flat.push_back(kEnd);
      }
    }
  }

  bool match(int cls, uint32_t cp) const {
    const auto& r = classes[cls];
    auto it = std::upper_bound(r.begin(), r.end(), std::make_pair(cp, UINT32_MAX));
    if (it == r.begin()) return false;
    --it;
    return it->first <= cp && cp <= it->second;
  }
};

struct Vocab {
  struct Node {
    std::vector<std::pair<uint32_t, int>> kids;   // sorted by code point
    std::vector<int> toks;                         // token ids whose text ends here
  };
  std::vector<Node> nodes;
  std::vector<std::vector<uint32_t>> text;
  uint64_t serial;                                 // mask-cache key (never reused)

  explicit Vocab(std::vector<std::vector<uint32_t>> toks) : text(std::move(toks)) {
    static std::atomic<uint64_t> next{1};
    serial = next.fetch_add(1);
    nodes.emplace_back();
    for (int id = 0; id < static_cast<int>(text.size()); ++id) {
      const auto& t = text[id];
      if (t.empty()) continue;                     // special tokens: never grammar text
      int n = 0;
      for (uint32_t cp : t) {
        auto& k = nodes[n].kids;
        auto it = std::lower_bound(k.begin(), k.end(), std::make_pair(cp, INT_MIN));
        if (it != k.end() && it->first == cp) {
          n = it->second;
        } else {
          const int c = static_cast<int>(nodes.size());
          k.insert(it, {cp, c});
          nodes.emplace_back();
          n = c;
        }
      }
      nodes[n].toks.push_back(id);
    }
  }
  int size() const { return static_cast<int>(text.size()); }
};

// Stack cells, stack sets and the lazy stack-set automaton, shared by every matcher of one
// grammar (engine/grammar.py caches grammars by text), so a state's token mask is computed once
// per process, like the regex FSM's DFA states.
class Automaton {
 public:
  explicit Automaton(std::shared_ptr<Grammar> g) : g_(std::move(g)) {
    sets_.push_back({});                         // set 0: dead
    set_ids_.emplace(std::vector<int>{}, 0);
    std::vector<int> init;
    for (int a : g_->alts[g_->start]) expand(push(a, -1), init, 0);
    start_ = intern_set(std::move(init));
  }

  int start() const { return start_; }
  bool accepting(int s) const { return !sets_[s].empty() && sets_[s].front() == -1; }
  bool can_continue(int s) const { return !sets_[s].empty() && sets_[s].back() != -1; }
  int num_stacks(int s) const { return static_cast<int>(sets_[s].size()); }
  size_t num_states() const { return sets_.size(); }

  int step(int s, uint32_t cp) {
    const uint64_t key = (static_cast<uint64_t>(s) << 21) | cp;
    auto it = trans_.find(key);
    if (it != trans_.end()) return it->second;
    std::vector<int> out;
    const std::vector<int> cur = sets_[s];       // copy: interning may grow sets_
    for (int st : cur) {
      if (st == -1) continue;
      const int pos = cells_[st].first;
      if (g_->match(g_->flat[pos], cp)) expand(push(pos + 1, cells_[st].second), out, 0);
    }
    const int r = intern_set(std::move(out));
    trans_.emplace(key, r);
    return r;
  }

  // bool mask over the vocabulary (1 = token text keeps some stack alive), cached per state.
  std::shared_ptr<const std::vector<uint8_t>> mask(int s, const Vocab& v) {
    const auto key = std::make_pair(v.serial, s);
    auto it = masks_.find(key);
    if (it != masks_.end()) return it->second;
    auto m = std::make_shared<std::vector<uint8_t>>(v.size(), 0);
    walk(v, 0, s, *m);
    if (masks_.size() >= kMaxMemo) masks_.clear();
    masks_.emplace(key, m);
    return m;
  }

  std::mutex mu;

 private:
  int push(int pos, int parent) {
    const uint64_t key = (static_cast<uint64_t>(static_cast<uint32_t>(pos)) << 32) |
                         static_cast<uint32_t>(parent + 1);
    auto it = intern_.find(key);
    if (it != intern_.end()) return it->second;
    const int id = static_cast<int>(cells_.size());
    cells_.push_back({pos, parent});
    intern_.emplace(key, id);
    return id;
  }

  // Close a stack under rule expansion / alternative completion; tops land on classes.
  void expand(int st, std::vector<int>& out, int depth) {
    if (depth > kMaxExpandDepth) throw std::runtime_error("grammar: expansion too deep (left recursion?)");
    for (;;) {
      if (st == -1) { out.push_back(-1); return; }
      const int pos = cells_[st].first, parent = cells_[st].second;
      const int s = g_->flat[pos];
      if (s == kEnd) { st = parent; continue; }     // alternative done: return
      if (s >= 0) { out.push_back(st); return; }
      const int r = -s - 1;
      const int ret = g_->flat[pos + 1] == kEnd ? parent : push(pos + 1, parent);   // tail call
      for (int a : g_->alts[r]) expand(push(a, ret), out, depth + 1);
      return;
    }
  }

  int intern_set(std::vector<int> v) {
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    if (v.size() > kMaxStacks) throw std::runtime_error("grammar: too ambiguous (stack set overflow)");
    auto it = set_ids_.find(v);
    if (it != set_ids_.end()) return it->second;
    const int id = static_cast<int>(sets_.size());
    sets_.push_back(v);
    set_ids_.emplace(std::move(v), id);
    return id;
  }

  void walk(const Vocab& v, int node, int s, std::vector<uint8_t>& m) {
    for (const auto& [cp, child] : v.nodes[node].kids) {
      const int ns = step(s, cp);
      if (ns == 0) continue;
      for (int t : v.nodes[child].toks) m[t] = 1;
      if (can_continue(ns) && !v.nodes[child].kids.empty()) walk(v, child, ns, m);
    }
  }

  std::shared_ptr<Grammar> g_;
  std::vector<std::pair<int, int>> cells_;        // interned stack cells (pos, parent)
  std::unordered_map<uint64_t, int> intern_;
  std::vector<std::vector<int>> sets_;            // interned stack sets (sorted; -1 = complete)
  std::map<std::vector<int>, int> set_ids_;
  std::unordered_map<uint64_t, int> trans_;       // (set, code point) -> set
  std::map<std::pair<uint64_t, int>, std::shared_ptr<const std::vector<uint8_t>>> masks_;
  int start_ = 0;
};

class Matcher {
 public:
  Matcher(std::shared_ptr<Automaton> a, std::shared_ptr<Vocab> v)
      : a_(std::move(a)), v_(std::move(v)), cur_(a_->start()) {}

  py::array_t<uint8_t> mask() {
    std::shared_ptr<const std::vector<uint8_t>> m;
    {
      py::gil_scoped_release nogil;
      std::lock_guard<std::mutex> lk(a_->mu);
      m = a_->mask(cur_, *v_);
    }
    py::array_t<uint8_t> out(static_cast<py::ssize_t>(m->size()));
    std::copy(m->begin(), m->end(), out.mutable_data());
    return out;
  }

  std::vector<int> allowed() {
    std::lock_guard<std::mutex> lk(a_->mu);
    const auto m = a_->mask(cur_, *v_);
    std::vector<int> ids;
    for (int i = 0; i < static_cast<int>(m->size()); ++i)
      if ((*m)[i]) ids.push_back(i);
    return ids;
  }

  bool advance_token(int id) {
    if (id < 0 || id >= v_->size() || v_->text[id].empty()) return false;
    return advance_text(v_->text[id]);
  }

  bool advance_text(const std::vector<uint32_t>& cps) {
    std::lock_guard<std::mutex> lk(a_->mu);
    int s = cur_;
    for (uint32_t cp : cps) {
      s = a_->step(s, cp);
      if (s == 0) return false;
    }
    cur_ = s;
    return true;
  }

  int state() const { return cur_; }
  bool accepting() const { return a_->accepting(cur_); }
  bool can_continue() const { return a_->can_continue(cur_); }
  int num_stacks() const { return a_->num_stacks(cur_); }

 private:
  std::shared_ptr<Automaton> a_;
  std::shared_ptr<Vocab> v_;
  int cur_;
};

}  // namespace

void register_grammar(py::module_& m) {
  py::class_<Grammar, std::shared_ptr<Grammar>>(m, "GrammarRules")
      .def(py::init<std::vector<std::vector<std::pair<uint32_t, uint32_t>>>,
                    const std::vector<std::vector<std::vector<int>>>&, int>(),
           py::arg("classes"), py::arg("rules"), py::arg("start"))
      .def_property_readonly("num_rules", [](const Grammar& g) { return g.alts.size(); });
  py::class_<Automaton, std::shared_ptr<Automaton>>(m, "Grammar")
      .def(py::init([](std::vector<std::vector<std::pair<uint32_t, uint32_t>>> classes,
                       const std::vector<std::vector<std::vector<int>>>& rules, int start) {
             return std::make_shared<Automaton>(
                 std::make_shared<Grammar>(std::move(classes), rules, start));
           }),
           py::arg("classes"), py::arg("rules"), py::arg("start"))
      .def_property_readonly("num_states", [](Automaton& a) {
        std::lock_guard<std::mutex> lk(a.mu);
        return a.num_states();
      });
  py::class_<Vocab, std::shared_ptr<Vocab>>(m, "GrammarVocab")
      .def(py::init<std::vector<std::vector<uint32_t>>>(), py::arg("token_codepoints"))
      .def_property_readonly("size", &Vocab::size)
      .def_property_readonly("num_nodes", [](const Vocab& v) { return v.nodes.size(); });
  py::class_<Matcher>(m, "GrammarMatcher")
      .def(py::init<std::shared_ptr<Automaton>, std::shared_ptr<Vocab>>())
      .def("mask", &Matcher::mask)
      .def("allowed", &Matcher::allowed, py::call_guard<py::gil_scoped_release>())
      .def("advance_token", &Matcher::advance_token)
      .def("advance_text", &Matcher::advance_text)
      .def("state", &Matcher::state)
      .def("accepting", &Matcher::accepting)
      .def("can_continue", &Matcher::can_continue)
      .def("num_stacks", &Matcher::num_stacks);
}
