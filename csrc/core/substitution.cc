// Graph substitutions: loader for the reference's rule-collection JSON format
// (substitutions/graph_subst_3_v2.json; reference src/runtime/substitution_loader.cc) and a
// backtracking subgraph matcher (reference GraphXfer::run / can_match, substitution.cc).
#include <fstream>
#include <set>
#include <sstream>
#include <stdexcept>

#include "json.h"
#include "pcg.h"

namespace ffcore {

std::vector<Rule> load_rules(const std::string& path) {
  std::ifstream f(path);
  if (!f) throw std::runtime_error("cannot open rule file " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string text = ss.str();
  Json j = parse_json(text);
  const Json& rules = j.at("rule");
  std::vector<Rule> out;
  out.reserve(rules.arr.size());
  auto op_of = [](const Json& o) {
    RuleOp r;
    r.type = o.at("type").as_str();
    for (const Json& t : o.at("input").arr) r.inputs.push_back({t.at("opId").as_int(), t.at("tsId").as_int()});
    for (const Json& pm : o.at("para").arr) r.params.push_back({pm.at("key").as_str(), pm.at("value").as_int()});
    return r;
  };
  for (const Json& r : rules.arr) {
    Rule x;
    if (const Json* nm = r.find("name")) x.name = nm->as_str();
    for (const Json& o : r.at("srcOp").arr) x.src.push_back(op_of(o));
    for (const Json& o : r.at("dstOp").arr) x.dst.push_back(op_of(o));
    for (const Json& m : r.at("mappedOutput").arr)
      x.mapped.push_back({m.at("srcOpId").as_int(), m.at("srcTsId").as_int(), m.at("dstOpId").as_int(),
                          m.at("dstTsId").as_int()});
    out.push_back(std::move(x));
  }
  return out;
}

namespace {

struct Matcher {
  const Rule& r;
  const std::vector<GNode>& g;
  std::vector<std::vector<std::pair<int, int>>> consumers;  // per graph node: (consumer, input slot)
  std::vector<int> assign;
  std::map<int, std::pair<int, int>> ext;
  std::vector<Match> out;
  int max_matches;

  Matcher(const Rule& r_, const std::vector<GNode>& g_, int mm) : r(r_), g(g_), max_matches(mm) {
    consumers.resize(g.size());
    for (size_t i = 0; i < g.size(); ++i)
      for (size_t s = 0; s < g[i].inputs.size(); ++s)
        if (g[i].inputs[s].first >= 0) consumers[g[i].inputs[s].first].push_back({(int)i, (int)s});
    assign.assign(r.src.size(), -1);
  }

  bool params_ok(const RuleOp& ro, const GNode& gn) const {
    for (const RuleParam& p : ro.params) {
      auto it = gn.params.find(p.key);
      if (it == gn.params.end() || it->second != p.value) return false;
    }
    return true;
  }

  bool closed() const {
    // matched intermediate outputs that are not mapped to the replacement may only feed matched ops
    std::set<int> in_match(assign.begin(), assign.end());
    for (size_t k = 0; k < assign.size(); ++k) {
      const int gn = assign[k];
      for (int t = 0; t < g[gn].num_outputs; ++t) {
        bool mapped = false;
        for (auto& m : r.mapped)
          if (m.src_op == (int)k && m.src_ts == t) mapped = true;
        if (mapped) continue;
        for (auto& c : consumers[gn])
          if (g[c.first].inputs[c.second].second == t && !in_match.count(c.first)) return false;
      }
    }
    return true;
  }

  void rec(size_t i) {
    if ((int)out.size() >= max_matches) return;
    if (i == r.src.size()) {
      if (closed()) out.push_back({assign, ext});
      return;
    }
    const RuleOp& ro = r.src[i];
    for (int gi = 0; gi < (int)g.size(); ++gi) {
      const GNode& gn = g[gi];
      if (gn.type != ro.type || gn.inputs.size() != ro.inputs.size() || !params_ok(ro, gn)) continue;
      if (std::find(assign.begin(), assign.end(), gi) != assign.end()) continue;
      auto saved_ext = ext;
      bool ok = true;
      for (size_t s = 0; s < ro.inputs.size() && ok; ++s) {
        const RuleTensor& t = ro.inputs[s];
        const auto& gin = gn.inputs[s];
        if (t.op_id >= 0) {
          ok = assign[t.op_id] >= 0 && gin.first == assign[t.op_id] && gin.second == t.ts_id;
        } else {
          auto it = ext.find(t.op_id);
          if (it == ext.end()) ext[t.op_id] = gin;
          else ok = it->second == gin;
        }
      }
      if (ok) {
        assign[i] = gi;
        rec(i + 1);
        assign[i] = -1;
      }
      ext = saved_ext;
      if ((int)out.size() >= max_matches) return;
    }
  }
};

}  // namespace

std::vector<Match> match_rule(const Rule& r, const std::vector<GNode>& g, int max_matches) {
  Matcher m(r, g, max_matches);
  // rule ops may reference later ops' outputs only if listed in order; reference rules are
  // topologically ordered, which the sequential assignment relies on
  m.rec(0);
  return m.out;
}

}  // namespace ffcore
