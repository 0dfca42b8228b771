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
//   * allowed(): one depth-first walk of the vocabulary trie carrying the stack set -- shared
//     prefixes are stepped once, a branch dies as soon as its set empties -- memoised per
//     stack set (a JSON string body or a list separator recurs many times per request).
//
// Left recursion is rejected when the grammar is compiled (engine/grammar.py); the expansion
// additionally caps its depth so a hand-built grammar cannot loop.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <unordered_map>
#include <utility>
#include <vector>

namespace py = pybind11;

namespace {

constexpr int kEnd = INT_MIN;
constexpr size_t kMaxStacks = 4096;
constexpr int kMaxExpandDepth = 4096;
constexpr size_t kMaxMemo = 512;

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

  explicit Vocab(std::vector<std::vector<uint32_t>> toks) : text(std::move(toks)) {
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

class Matcher {
 public:
  Matcher(std::shared_ptr<Grammar> g, std::shared_ptr<Vocab> v) : g_(std::move(g)), v_(std::move(v)) {
    for (int a : g_->alts[g_->start]) expand(push(a, -1), cur_, 0);
    normalise(cur_);
  }

  std::vector<int> allowed() {
    auto it = memo_.find(cur_);
    if (it != memo_.end()) return it->second;
    std::vector<int> out;
    walk(0, cur_, out);
    std::sort(out.begin(), out.end());
    if (memo_.size() >= kMaxMemo) memo_.clear();
    memo_.emplace(cur_, out);
    return out;
  }

  bool advance_token(int id) {
    if (id < 0 || id >= v_->size() || v_->text[id].empty()) return false;
    std::vector<int> s = cur_;
    for (uint32_t cp : v_->text[id]) {
      s = step(s, cp);
      if (s.empty()) return false;
    }
    cur_ = std::move(s);
    return true;
  }

  bool advance_text(const std::vector<uint32_t>& cps) {
    std::vector<int> s = cur_;
    for (uint32_t cp : cps) {
      s = step(s, cp);
      if (s.empty()) return false;
    }
    cur_ = std::move(s);
    return true;
  }

  bool accepting() const { return !cur_.empty() && cur_.front() == -1; }
  bool can_continue() const { return !cur_.empty() && cur_.back() != -1; }
  int num_stacks() const { return static_cast<int>(cur_.size()); }

 private:
  int push(int pos, int parent) {
    const uint64_t key = (static_cast<uint64_t>(static_cast<uint32_t>(pos)) << 32) |
                         static_cast<uint32_t>(parent + 1);
    auto it = intern_.find(key);
    if (it != intern_.end()) return it->second;
    const int id = static_cast<int>(nodes_.size());
    nodes_.push_back({pos, parent});
    intern_.emplace(key, id);
    return id;
  }

  // Close a stack under rule expansion / alternative completion; tops land on classes.
  void expand(int st, std::vector<int>& out, int depth) {
    if (depth > kMaxExpandDepth) throw std::runtime_error("grammar: expansion too deep (left recursion?)");
    for (;;) {
      if (st == -1) { out.push_back(-1); return; }
      const int pos = nodes_[st].first, parent = nodes_[st].second;
      const int s = g_->flat[pos];
      if (s == kEnd) { st = parent; continue; }     // alternative done: return
      if (s >= 0) { out.push_back(st); return; }
      const int r = -s - 1;
      const int ret = g_->flat[pos + 1] == kEnd ? parent : push(pos + 1, parent);   // tail call
      for (int a : g_->alts[r]) expand(push(a, ret), out, depth + 1);
      return;
    }
  }

  static void normalise(std::vector<int>& v) {
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    if (v.size() > kMaxStacks) throw std::runtime_error("grammar: too ambiguous (stack set overflow)");
  }

  std::vector<int> step(const std::vector<int>& set, uint32_t cp) {
    std::vector<int> out;
    for (int st : set) {
      if (st == -1) continue;
      const int pos = nodes_[st].first;
      if (g_->match(g_->flat[pos], cp)) expand(push(pos + 1, nodes_[st].second), out, 0);
    }
    normalise(out);
    return out;
  }

  void walk(int node, const std::vector<int>& set, std::vector<int>& out) {
    for (const auto& [cp, child] : v_->nodes[node].kids) {
      std::vector<int> ns = step(set, cp);
      if (ns.empty()) continue;
      const auto& t = v_->nodes[child].toks;
      out.insert(out.end(), t.begin(), t.end());
      if (ns.back() != -1 && !v_->nodes[child].kids.empty()) walk(child, ns, out);
    }
  }

  std::shared_ptr<Grammar> g_;
  std::shared_ptr<Vocab> v_;
  std::vector<std::pair<int, int>> nodes_;        // interned stack cells (pos, parent)
  std::unordered_map<uint64_t, int> intern_;
  std::vector<int> cur_;                          // sorted stack ids; -1 = complete
  std::map<std::vector<int>, std::vector<int>> memo_;
};

}  // namespace

void register_grammar(py::module_& m) {
  py::class_<Grammar, std::shared_ptr<Grammar>>(m, "Grammar")
      .def(py::init<std::vector<std::vector<std::pair<uint32_t, uint32_t>>>,
                    const std::vector<std::vector<std::vector<int>>>&, int>(),
           py::arg("classes"), py::arg("rules"), py::arg("start"))
      .def_property_readonly("num_rules", [](const Grammar& g) { return g.alts.size(); });
  py::class_<Vocab, std::shared_ptr<Vocab>>(m, "GrammarVocab")
      .def(py::init<std::vector<std::vector<uint32_t>>>(), py::arg("token_codepoints"))
      .def_property_readonly("size", &Vocab::size)
      .def_property_readonly("num_nodes", [](const Vocab& v) { return v.nodes.size(); });
  py::class_<Matcher>(m, "GrammarMatcher")
      .def(py::init<std::shared_ptr<Grammar>, std::shared_ptr<Vocab>>())
      .def("allowed", &Matcher::allowed, py::call_guard<py::gil_scoped_release>())
      .def("advance_token", &Matcher::advance_token)
      .def("advance_text", &Matcher::advance_text)
      .def("accepting", &Matcher::accepting)
      .def("can_continue", &Matcher::can_continue)
      .def("num_stacks", &Matcher::num_stacks);
}
