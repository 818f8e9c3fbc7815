#include "framework/framework.h"

#include <algorithm>
#include <atomic>
#include <stdexcept>

#include "scheduler/metrics.h"
#include "scheduler/queue.h"

namespace xsched {

namespace {
const std::pair<const char*, uint32_t> kPointNames[] = {
    {"queueSort", kQueueSort}, {"preFilter", kPreFilter}, {"filter", kFilter},   {"postFilter", kPostFilter},
    {"preScore", kPreScore},   {"score", kScore},         {"reserve", kReserve}, {"permit", kPermit},
    {"preBind", kPreBind},     {"bind", kBind},           {"postBind", kPostBind},
};
}  // namespace

const char* ext_point_name(uint32_t p) {
  for (const auto& kv : kPointNames)
    if (kv.second == p) return kv.first;
  return "unknown";
}

uint32_t ext_point_from_name(const std::string& n) {
  for (const auto& kv : kPointNames)
    if (n == kv.first) return kv.second;
  return 0;
}

// ------------------------------------------------------------ Registry ----
Registry& Registry::global() {
  static Registry* r = new Registry();
  return *r;
}

void Registry::add(const std::string& name, PluginFactory f) { factories_[name] = std::move(f); }

PluginPtr Registry::make(const std::string& name, const Json& args, Handle& h) const {
  auto it = factories_.find(name);
  if (it == factories_.end()) throw std::runtime_error("plugin \"" + name + "\" does not exist");
  return it->second(args, h);
}

std::vector<std::string> Registry::names() const {
  std::vector<std::string> out;
  for (const auto& kv : factories_) out.push_back(kv.first);
  std::sort(out.begin(), out.end());
  return out;
}

void default_normalize_score(int64_t max_priority, bool reverse, std::vector<NodeScore>& scores) {
  int64_t max_count = 0, min_count = 0;
  for (const auto& s : scores) {
    max_count = std::max(max_count, s.score);
    min_count = std::min(min_count, s.score);
  }
  if (max_count == 0) {
    if (reverse)
      for (auto& s : scores) s.score = max_priority;
    return;
  }
  // Raw scores are mostly small counts (free GPUs, matching pods): one
  // division per distinct value instead of one per node.
  if (min_count >= 0 && max_count < 256 && static_cast<size_t>(max_count) * 2 < scores.size()) {
    int64_t table[256];
    for (int64_t v = 0; v <= max_count; ++v) {
      const int64_t sc = max_priority * v / max_count;
      table[v] = reverse ? max_priority - sc : sc;
    }
    for (auto& s : scores) s.score = table[s.score];
    return;
  }
  if (min_count >= 0 && max_priority > 0 && max_count <= (int64_t{1} << 52) / max_priority) {
    // Non-negative numerators below 2^52 (exact as doubles): a double
    // reciprocal is within one of the quotient, and one correction step
    // each way makes it exact.
    const double inv = 1.0 / static_cast<double>(max_count);
    for (auto& s : scores) {
      const int64_t num = max_priority * s.score;
      int64_t q = static_cast<int64_t>(static_cast<double>(num) * inv);
      if (q * max_count > num) --q;
      else if ((q + 1) * max_count <= num) ++q;
      s.score = reverse ? max_priority - q : q;
    }
    return;
  }
  for (auto& s : scores) {
    int64_t sc = max_priority * s.score / max_count;
    if (reverse) sc = max_priority - sc;
    s.score = sc;
  }
}

// ------------------------------------------------------- ProfileConfig ----
ProfileConfig ProfileConfig::from_json(const Json& j) {
  ProfileConfig c;
  c.scheduler_name = j["schedulerName"].str_or(kDefaultSchedulerName);
  for (const auto& kv : j["plugins"].members()) {
    uint32_t pt = ext_point_from_name(kv.first);
    if (!pt) throw std::runtime_error("unknown extension point " + kv.first);
    auto& vec = c.enabled[pt];
    for (const auto& e : kv.second.items()) {
      std::string name = e.is_string() ? e.as_string() : e["name"].as_string();
      vec.push_back(name);
      if (pt == kScore) c.score_weights[name] = e.is_object() ? std::max<int64_t>(1, e["weight"].as_int(1)) : 1;
    }
  }
  for (const auto& kv : j["pluginConfig"].members()) c.plugin_args[kv.first] = kv.second;
  c.percentage_of_nodes_to_score = static_cast<int>(j["percentageOfNodesToScore"].as_int(0));
  c.run_all_filters = j["runAllFilters"].as_bool(false);
  return c;
}

// ----------------------------------------------------------- Framework ----
Framework::Framework(const ProfileConfig& cfg, Handle handle) : cfg_(cfg), handle_(handle) {
  handle_.framework = this;
  auto& reg = Registry::global();
  for (const auto& [pt, names] : cfg_.enabled) {
    for (const auto& name : names) {
      PluginPtr p;
      auto it = by_name_.find(name);
      if (it != by_name_.end()) {
        p = it->second;
      } else {
        auto ait = cfg_.plugin_args.find(name);
        p = reg.make(name, ait == cfg_.plugin_args.end() ? Json::object() : ait->second, handle_);
        by_name_[name] = p;
        all_.push_back(p);
      }
      if (!(p->points() & pt))
        throw std::runtime_error("plugin \"" + name + "\" does not extend " + ext_point_name(pt) + " plugin");
      auto& chain = chain_[pt];
      if (std::find(chain.begin(), chain.end(), p) != chain.end())
        throw std::runtime_error("plugin \"" + name + "\" already registered as \"" + ext_point_name(pt) + "\"");
      chain.push_back(p);
      if (pt == kScore) scorers_.emplace_back(p, cfg_.score_weights.count(name) ? cfg_.score_weights[name] : 1);
    }
  }
  auto qs = chain_.find(kQueueSort);
  if (qs == chain_.end() || qs->second.size() != 1)
    throw std::runtime_error("one queue sort plugin required for profile " + cfg_.scheduler_name);
  queue_sort_ = qs->second.front();
  auto bd = chain_.find(kBind);
  if (bd == chain_.end() || bd->second.empty())
    throw std::runtime_error("at least one bind plugin is needed for profile " + cfg_.scheduler_name);
  for (const auto& p : all_) {
    for (const auto& k : p->watched_kinds()) kind_watchers_[k].push_back(p);
    if (p->wants_capacity_events()) capacity_watchers_.push_back(p);
  }
}

Framework::~Framework() = default;

PluginPtr Framework::plugin(const std::string& name) const {
  auto it = by_name_.find(name);
  return it == by_name_.end() ? nullptr : it->second;
}

bool Framework::has(uint32_t point) const {
  auto it = chain_.find(point);
  return it != chain_.end() && !it->second.empty();
}

bool Framework::less(const QueuedPodInfo& a, const QueuedPodInfo& b) const { return queue_sort_->less(a, b); }

void Framework::record(const char* point, const Status& st, int64_t start_us, CycleState& s) {
  if (!s.record_metrics || !handle_.metrics) return;
  double d = static_cast<double>(handle_.clock->now_us() - start_us) / 1e6;
  handle_.metrics
      ->histogram("scheduler_framework_extension_point_duration_seconds",
                  std::string("extension_point=\"") + point + "\",profile=\"" + cfg_.scheduler_name + "\",status=\"" +
                      code_name(st.code()) + "\"")
      .observe(d);
}

Status Framework::run_pre_filter(CycleState& s, const Pod& p) {
  int64_t t0 = s.record_metrics ? handle_.clock->now_us() : 0;
  s.filter_skip = 0;
  if (auto fit = chain_.find(kFilter); fit != chain_.end() && fit->second.size() <= 64)
    for (size_t k = 0; k < fit->second.size(); ++k)
      if (fit->second[k]->skip_filter(p)) s.filter_skip |= uint64_t{1} << k;
  auto it = chain_.find(kPreFilter);
  if (it != chain_.end()) {
    for (const auto& pl : it->second) {
      Status st = pl->pre_filter(s, p);
      if (!st.is_success()) {
        st.with_plugin(pl->name_ptr());
        if (st.code() == Code::Error) {
          Status e(Code::Error, "running PreFilter plugin \"" + pl->name() + "\": " + st.message());
          e.with_plugin(pl->name_ptr());
          record("PreFilter", e, t0, s);
          return e;
        }
        record("PreFilter", st, t0, s);
        return st;
      }
    }
  }
  record("PreFilter", Status(), t0, s);
  return {};
}

Status Framework::run_pre_filter_add_pod(CycleState& s, const Pod& to_schedule, const PodPtr& to_add,
                                         const NodeInfo& ni) {
  auto it = chain_.find(kPreFilter);
  if (it == chain_.end()) return {};
  for (const auto& pl : it->second) {
    if (!pl->has_pre_filter_extensions() || !pl->pre_filter_extension_affects(s, to_schedule, *to_add)) continue;
    Status st = pl->add_pod(s, to_schedule, to_add, ni);
    if (!st.is_success()) return Status(Code::Error, "running AddPod on PreFilter plugin " + pl->name() + ": " + st.message());
  }
  return {};
}

Status Framework::run_pre_filter_remove_pod(CycleState& s, const Pod& to_schedule, const PodPtr& to_remove,
                                            const NodeInfo& ni) {
  auto it = chain_.find(kPreFilter);
  if (it == chain_.end()) return {};
  for (const auto& pl : it->second) {
    if (!pl->has_pre_filter_extensions() || !pl->pre_filter_extension_affects(s, to_schedule, *to_remove)) continue;
    Status st = pl->remove_pod(s, to_schedule, to_remove, ni);
    if (!st.is_success())
      return Status(Code::Error, "running RemovePod on PreFilter plugin " + pl->name() + ": " + st.message());
  }
  return {};
}

bool Framework::pre_filter_extensions_affected(const CycleState& s, const Pod& to_schedule, const Pod& other,
                                               const std::string* except) const {
  auto it = chain_.find(kPreFilter);
  if (it == chain_.end()) return false;
  for (const auto& pl : it->second)
    if (pl->has_pre_filter_extensions() && !(except && pl->name() == *except) &&
        pl->pre_filter_extension_affects(s, to_schedule, other))
      return true;
  return false;
}

Status Framework::run_filter(CycleState& s, const Pod& p, const NodeInfo& ni) {
  auto it = chain_.find(kFilter);
  if (it == chain_.end()) return {};
  Status merged;
  bool failed = false;
  const uint64_t skip = s.filter_skip;
  for (size_t k = 0; k < it->second.size(); ++k) {
    if ((skip >> k) & 1u) continue;
    const auto& pl = it->second[k];
    Status st = pl->filter(s, p, ni);
    if (st.is_success()) continue;
    if (!st.is_unschedulable()) {
      Status e(Code::Error, "running \"" + pl->name() + "\" filter plugin: " + st.message());
      e.with_plugin(pl->name_ptr());
      return e;
    }
    st.with_plugin(pl->name_ptr());
    if (!cfg_.run_all_filters) return st;
    if (!failed) {
      merged = st;
      failed = true;
    }
  }
  return failed ? merged : Status();
}

Status Framework::run_filter_with_nominated_pods(CycleState& s, const Pod& p, const NodeInfo& ni) {
  return filter_with_nominated(s, p, ni, nullptr);
}

Status Framework::run_filter_with_nominated_pods_inplace(CycleState& s, const Pod& p, NodeInfo& ni) {
  return filter_with_nominated(s, p, ni, &ni);
}

uint64_t Framework::nominated_signature(const CycleState& s, const Pod& p, const NodeInfo& ni, bool* cacheable) const {
  *cacheable = true;
  if (!s.nominated || !ni.node) {
    *cacheable = false;  // no cycle view: nominations not pinned for this cycle
    return 1;
  }
  auto it = s.nominated->find(ni.name());
  if (it == s.nominated->end()) return 0;
  return nominated_signature(s, p, &it->second, cacheable);
}

uint64_t Framework::nominated_signature(const CycleState& s, const Pod& p, const std::vector<PodPtr>* list,
                                        bool* cacheable) const {
  *cacheable = true;
  if (!list) return 0;
  uint64_t h = 1469598103934665603ULL;
  bool any = false;
  for (const auto& np : *list) {
    if (np->priority < p.priority || np->uid() == p.uid()) continue;
    any = true;
    uint64_t x = std::hash<std::string>{}(np->uid()) ^ (np->template_hash * 0x9E3779B97F4A7C15ULL) ^
                 (static_cast<uint64_t>(static_cast<uint32_t>(np->priority)) << 17);
    h = (h ^ x) * 1099511628211ULL;
    if (pre_filter_extensions_affected(s, p, *np)) *cacheable = false;
  }
  return any ? (h ? h : 1) : 0;
}

Status Framework::filter_with_nominated(CycleState& s, const Pod& p, const NodeInfo& ni, NodeInfo* inplace) {
  Status st;
  bool pods_added = false;
  // In place: the nominated pods join `inplace` for the first pass and leave
  // it before the second (and on every return), instead of a copy of it.
  thread_local std::vector<PodPtr> added_here;
  struct Undo {
    NodeInfo* ni;
    size_t base;  // re-entrancy safe: only this call's tail is undone
    void operator()() {
      if (!ni) return;
      while (added_here.size() > base) {
        ni->remove_pod(added_here.back()->uid());
        added_here.pop_back();
      }
    }
    ~Undo() { (*this)(); }
  } undo{inplace, added_here.size()};
  for (int i = 0; i < 2; ++i) {
    CycleState* state_to_use = &s;
    const NodeInfo* ni_to_use = &ni;
    std::shared_ptr<CycleState> state_out;
    // addNominatedPods works on a copy of the node: this thread's scratch,
    // whose storage is reused from call to call (no allocation per node).
    thread_local NodeInfo scratch;
    NodeInfo* ni_out = nullptr;
    if (i == 0) {
      std::vector<PodPtr> live;
      const std::vector<PodPtr>* nominated = &live;
      if (!ni.node) {
      } else if (s.nominated) {
        auto it = s.nominated->find(ni.name());
        if (it != s.nominated->end()) nominated = &it->second;
      } else if (handle_.nominator && !handle_.nominator->empty()) {
        live = handle_.nominator->nominated_pods_for_node(ni.name());
      }
      for (const auto& np : *nominated) {
        if (np->priority < p.priority || np->uid() == p.uid()) continue;
        if (!ni_out) {
          if (inplace) {
            ni_out = inplace;
          } else {
            scratch = ni;
            ni_out = &scratch;
          }
        }
        ni_out->add_pod(np);
        if (inplace) added_here.push_back(np);
        pods_added = true;
        // addNominatedPods clones the CycleState for the PreFilter AddPod
        // extensions; a nominated pod none of them reacts to leaves the state
        // as it is, so the clone waits for the first one that does (the
        // skipped pods changed nothing it would have carried).
        if (!pre_filter_extensions_affected(s, p, *np)) continue;
        if (!state_out) state_out = s.clone();
        Status ast = run_pre_filter_add_pod(*state_out, p, np, *ni_out);
        if (!ast.is_success()) return ast;
      }
      if (pods_added) {
        if (state_out) state_to_use = state_out.get();
        ni_to_use = ni_out;
      }
    } else if (!pods_added || !st.is_success()) {
      break;
    }
    st = run_filter(*state_to_use, p, *ni_to_use);
    if (!st.is_success() && !st.is_unschedulable()) return st;
    if (inplace) undo();  // the second pass sees the node without them
  }
  return st;
}

std::pair<PostFilterResult, Status> Framework::run_post_filter(CycleState& s, const Pod& p, const NodeStatusMap& m) {
  int64_t t0 = s.record_metrics ? handle_.clock->now_us() : 0;
  auto it = chain_.find(kPostFilter);
  Status last(Code::Unschedulable);
  if (it != chain_.end()) {
    for (const auto& pl : it->second) {
      auto [res, st] = pl->post_filter(s, p, m);
      if (st.is_success()) {
        record("PostFilter", st, t0, s);
        return {res, st};
      }
      if (!st.is_unschedulable()) {
        record("PostFilter", st, t0, s);
        return {PostFilterResult{}, Status(Code::Error, st.message()).with_plugin(pl->name_ptr())};
      }
      last = st;
      last.with_plugin(pl->name_ptr());
    }
  }
  record("PostFilter", last, t0, s);
  return {PostFilterResult{}, last};
}

Status Framework::run_pre_score(CycleState& s, const Pod& p, const NodeList& nodes) {
  auto it = chain_.find(kPreScore);
  if (it == chain_.end()) return {};
  for (const auto& pl : it->second) {
    Status st = pl->pre_score(s, p, nodes);
    if (!st.is_success()) return Status(Code::Error, "running PreScore plugin " + pl->name() + ": " + st.message());
  }
  return {};
}

bool Framework::filters_node_local(const Pod& p, const Snapshot& snap) const {
  auto it = chain_.find(kFilter);
  if (it == chain_.end()) return true;
  for (const auto& pl : it->second)
    if (!pl->skip_filter(p) && !pl->filter_node_local(p, snap)) return false;
  return true;
}

std::vector<char> Framework::local_scorers(const Pod& p, const Snapshot& snap) const {
  std::vector<char> out;
  local_scorers(p, snap, out);
  return out;
}

void Framework::local_scorers(const Pod& p, const Snapshot& snap, std::vector<char>& out) const {
  out.assign(scorers_.size(), 0);
  bool any = false;
  for (size_t k = 0; k < scorers_.size(); ++k) {
    out[k] = scorers_[k].first->score_node_local(p, snap) ? 1 : 0;
    any = any || out[k];
  }
  if (!any) out.clear();
}

Status Framework::run_score(CycleState& s, const Pod& p, const NodeList& nodes,
                            std::vector<NodeScore>& total, ScoreBreakdown* breakdown, EqScoreCache* eq) {
  int64_t t0 = s.record_metrics ? handle_.clock->now_us() : 0;
  size_t n = nodes.size();
  total.resize(n);
  for (size_t i = 0; i < n; ++i) total[i].score = 0;
  if (breakdown)
    for (size_t i = 0; i < n; ++i) total[i].name = &nodes[i]->name();
  if (scorers_.empty()) return {};
  // Per-plugin score rows are reused across cycles (no allocation or string
  // construction per plugin x node in steady state); every cell is written
  // below before it is read.
  // The rows are thread_local to the calling (scheduling) thread; the
  // node-parallel workers below must reach them through this reference, as
  // naming a thread_local inside the lambda would resolve to the worker's own.
  thread_local std::vector<std::vector<NodeScore>> per_rows;
  std::vector<std::vector<NodeScore>>& per = per_rows;
  if (per.size() < scorers_.size()) per.resize(scorers_.size());
  for (size_t k = 0; k < scorers_.size(); ++k) per[k].resize(n);
  // Plugins whose raw score is 0 on every node for this pod are skipped
  // (Plugin::score_all_zero); their rows are zero-filled so equivalence-cache
  // slots stay exact.
  thread_local std::vector<char> skip_rows;
  std::vector<char>& skip = skip_rows;
  skip.assign(scorers_.size(), 0);
  if (!breakdown && handle_.snapshot)
    for (size_t k = 0; k < scorers_.size(); ++k) skip[k] = scorers_[k].first->score_all_zero(p, *handle_.snapshot);
  std::atomic<bool> failed{false};
  std::string err;
  std::mutex err_mu;
  const size_t ns = scorers_.size();
  // The template's equivalence table, when every node's snapshot position is
  // known (ns <= 64: scorer sets are bitmasks). Per node it holds raw columns
  // valid at score_gen (the set `cols`) and the weighted sum of the plain
  // scorers (node-local, no normalization) over the set `plain_mask`.
  EqTable* table =
      eq && eq->table && eq->npos == n && eq->local.size() == ns && ns <= 64 ? eq->table : nullptr;
  if (table) table->ensure_scorers(ns);
  const int* tpos = table ? eq->pos : nullptr;
  uint64_t local_mask = 0;  // non-skipped node-local scorers
  if (table)
    for (size_t k = 0; k < ns; ++k)
      if (!skip[k] && eq->local[k]) local_mask |= 1ULL << k;
  // One node: every score plugin (raw scores; normalizers read the rows).
  auto score_node = [&](size_t i) {
    // Equivalence cache: node-local raw scores of this pod template on an
    // unchanged node are reused; the others are recomputed.
    const NodeInfo& ni = *nodes[i];
    const size_t pos = tpos ? static_cast<size_t>(tpos[i]) : 0;
    const bool hit = table && table->score_gen[pos] == ni.generation && (table->cols[pos] & local_mask) == local_mask;
    for (size_t k = 0; k < ns; ++k) {
      if (skip[k]) {
        per[k][i].score = 0;
        continue;
      }
      if (hit && eq->local[k]) {
        per[k][i].score = table->raw_at(k, pos);
        continue;
      }
      auto [sc, st] = scorers_[k].first->score(s, p, ni);
      if (!st.is_success()) {
        std::lock_guard<std::mutex> g(err_mu);
        err = "running Score plugin " + scorers_[k].first->name() + ": " + st.message();
        failed.store(true);
        return;
      }
      per[k][i].score = sc;
    }
    if (table && !hit) {
      for (size_t k = 0; k < ns; ++k)
        if ((local_mask >> k) & 1) table->raw_at(k, pos) = per[k][i].score;
      table->score_gen[pos] = ni.generation;
      table->cols[pos] = local_mask;
      table->plain_mask[pos] = 0;  // no sum here: a serial lookup with plain scorers misses
    }
  };
  // The serial path splits the local scorers into plain ones, summed per node
  // version once (a hit then costs one read for all of them), and row ones
  // (normalized per cycle), whose raw column is kept.
  uint64_t plain_mask = 0, row_mask = 0;
  thread_local std::vector<int64_t> plain_buf;
  std::vector<int64_t>& plain_tot = plain_buf;
  const bool inline_score = handle_.parallelizer->plan_inline(static_cast<int>(n), &score_site_);
  if (inline_score && table) {
    for (size_t k = 0; k < ns; ++k)
      if ((local_mask >> k) & 1) {
        if (!breakdown && !scorers_[k].first->has_normalize_score()) plain_mask |= 1ULL << k;
        else row_mask |= 1ULL << k;
      }
  }
  auto is_plain = [&](size_t k) { return (plain_mask >> k) & 1; };
  if (inline_score) {
    // Serial path, plugin-major: each scorer runs over every node that needs
    // it in one call (Plugin::score_many), equivalence-cache hits copied in.
    const int64_t s0 = Parallelizer::now_ns();
    thread_local std::vector<char> hit_buf;
    std::vector<char>& hit = hit_buf;
    thread_local std::vector<uint32_t> miss_buf;
    std::vector<uint32_t>& miss = miss_buf;  // indices of the nodes recomputed
    hit.assign(n, 0);
    miss.clear();
    if (plain_mask) plain_tot.assign(n, 0);
    bool any_hit = false;
    const bool have_gens = eq && eq->gen && eq->npos == n;
    if (table) {
      const int64_t* sgen = table->score_gen.data();
      const uint64_t* pm = table->plain_mask.data();
      const uint64_t* cm = table->cols.data();
      // Branch-free: hits and misses interleave unpredictably. Raw pointers:
      // through the thread_local vectors every char store could alias their
      // bookkeeping and forced a reload of the TLS slot per node.
      miss.resize(n);
      size_t nm = 0;
      char* hp = hit.data();
      uint32_t* mp = miss.data();
      const int64_t* eg = have_gens ? eq->gen : nullptr;
      const uint64_t pmask = plain_mask, rmask = row_mask;
      for (size_t i = 0; i < n; ++i) {
        const size_t pos = static_cast<size_t>(tpos[i]);
        const int64_t gen = eg ? eg[pos] : nodes[i]->generation;
        const bool h = (sgen[pos] == gen) & (pm[pos] == pmask) & ((cm[pos] & rmask) == rmask);
        hp[i] = h;
        mp[nm] = static_cast<uint32_t>(i);
        nm += !h;
      }
      miss.resize(nm);
      any_hit = nm < n;
    }
    // Hits: plain sums and row columns, copied for every node (a miss's
    // cells are overwritten below); skipped and plain scorers' rows are never
    // read, so they are not filled.
    if (any_hit) {
      if (plain_mask) {
        const int64_t* ps = table->plain_sum.data();
        for (size_t i = 0; i < n; ++i) plain_tot[i] = ps[tpos[i]];
      }
      for (size_t k = 0; k < ns; ++k) {  // column by column
        if (!((row_mask >> k) & 1)) continue;
        const int64_t* col = &table->raw[k * table->n];
        NodeScore* row = per[k].data();
        for (size_t i = 0; i < n; ++i) row[i].score = col[tpos[i]];
      }
    }
    for (size_t k = 0; k < ns; ++k) {
      std::vector<NodeScore>& row = per[k];
      if (skip[k]) continue;
      const bool reuse = any_hit && eq->local[k];
      Status st;
      if (reuse && miss.size() * 4 < n) {
        // Few misses: score just those (no pass over the hits).
        for (uint32_t i : miss) {
          auto [sc, one] = scorers_[k].first->score(s, p, *nodes[i]);
          if (!one.is_success()) {
            st = one;
            break;
          }
          row[i].score = sc;
        }
      } else {
        st = scorers_[k].first->score_many(s, p, nodes, reuse ? hit.data() : nullptr, row,
                                           (eq && eq->npos == n) ? eq->pos : nullptr);
      }
      if (!st.is_success()) {
        err = "running Score plugin " + scorers_[k].first->name() + ": " + st.message();
        failed.store(true);
        break;
      }
    }
    if (plain_mask && !failed.load())
      for (uint32_t i : miss) {
        int64_t sum = 0;
        for (size_t k = 0; k < ns; ++k) {
          if (!is_plain(k)) continue;
          const int64_t sc = per[k][i].score;
          if (sc > kMaxNodeScore || sc < kMinNodeScore) {
            err = "plugin \"" + scorers_[k].first->name() + "\" returns an invalid score " + std::to_string(sc) +
                  ", it should in the range of [0, 100] after normalizing";
            failed.store(true);
            break;
          }
          sum += sc * scorers_[k].second;
        }
        if (failed.load()) break;
        plain_tot[i] = sum;
      }
    if (table && !failed.load() && !miss.empty()) {
      for (size_t k = 0; k < ns; ++k) {  // row columns of the recomputed nodes
        if (!((row_mask >> k) & 1)) continue;
        int64_t* col = &table->raw[k * table->n];
        for (uint32_t i : miss) col[tpos[i]] = per[k][i].score;
      }
      for (uint32_t i : miss) {
        const size_t pos = static_cast<size_t>(tpos[i]);
        table->score_gen[pos] = have_gens ? eq->gen[pos] : nodes[i]->generation;
        table->cols[pos] = row_mask;
        table->plain_mask[pos] = plain_mask;
        table->plain_sum[pos] = plain_tot.size() == n && plain_mask ? plain_tot[i] : 0;
      }
    }
    Parallelizer::record_inline(&score_site_, Parallelizer::now_ns() - s0, static_cast<int>(n), static_cast<int>(n));
  } else {
    handle_.parallelizer->until_forked(static_cast<int>(n), [&](int i) { score_node(static_cast<size_t>(i)); },
                                       &failed, &score_site_);
  }
  if (failed.load()) return Status(Code::Error, err);
  int64_t skipped_total = 0;  // the skipped plugins' constant contribution
  for (size_t k = 0; k < scorers_.size(); ++k)
    if (skip[k]) skipped_total += scorers_[k].first->score_skip_value() * scorers_[k].second;
  if (plain_mask) {
    for (size_t i = 0; i < n; ++i) total[i].score += skipped_total + plain_tot[i];
  } else if (skipped_total) {
    for (size_t i = 0; i < n; ++i) total[i].score += skipped_total;
  }
  for (size_t k = 0; k < scorers_.size(); ++k) {
    if (skip[k] || is_plain(k)) continue;
    auto& pl = scorers_[k].first;
    if (pl->has_normalize_score()) {
      if (pl->normalize_uses_names())
        for (size_t i = 0; i < n; ++i) per[k][i].name = &nodes[i]->name();
      Status st = pl->normalize_score(s, p, per[k]);
      if (!st.is_success()) return Status(Code::Error, "running Normalize on Score plugin " + pl->name() + ": " + st.message());
    }
    int64_t w = scorers_[k].second;
    if (breakdown) {
      std::vector<int64_t> v(n);
      for (size_t i = 0; i < n; ++i) v[i] = per[k][i].score;
      breakdown->emplace_back(pl->name() + "*" + std::to_string(w), std::move(v));
    }
    for (size_t i = 0; i < n; ++i) {
      int64_t sc = per[k][i].score;
      if (sc > kMaxNodeScore || sc < kMinNodeScore)
        return Status(Code::Error, "plugin \"" + pl->name() + "\" returns an invalid score " + std::to_string(sc) +
                                       ", it should in the range of [0, 100] after normalizing");
      total[i].score += sc * w;
    }
  }
  record("Score", Status(), t0, s);
  return {};
}

Status Framework::run_reserve(CycleState& s, const PodPtr& p, const std::string& node) {
  auto it = chain_.find(kReserve);
  if (it == chain_.end()) return {};
  for (const auto& pl : it->second) {
    Status st = pl->reserve(s, p, node);
    if (!st.is_success()) {
      Status e(Code::Error, "running Reserve plugin \"" + pl->name() + "\": " + st.message());
      if (st.is_unschedulable()) e = Status(st.code(), st.message());
      e.with_plugin(pl->name_ptr());
      return e;
    }
  }
  return {};
}

void Framework::run_unreserve(CycleState& s, const PodPtr& p, const std::string& node) {
  auto it = chain_.find(kReserve);
  if (it == chain_.end()) return;
  for (auto rit = it->second.rbegin(); rit != it->second.rend(); ++rit) (*rit)->unreserve(s, p, node);
}

Status Framework::run_permit(CycleState& s, const PodPtr& p, const std::string& node,
                             std::function<void(const Status&)> on_done) {
  auto it = chain_.find(kPermit);
  if (it == chain_.end()) return {};
  std::map<std::string, int64_t> timeouts;
  for (const auto& pl : it->second) {
    auto [st, timeout] = pl->permit(s, p, node);
    if (st.is_success()) continue;
    if (st.is_unschedulable()) {
      st.with_plugin(pl->name_ptr());
      return st;
    }
    if (st.is_wait()) {
      timeouts[pl->name()] = std::min(std::max<int64_t>(timeout, 0), kMaxPermitTimeoutUs);
      continue;
    }
    return Status(Code::Error, "running Permit plugin " + pl->name() + ": " + st.message()).with_plugin(pl->name_ptr());
  }
  if (timeouts.empty()) return {};
  handle_.waiting_pods->add(p, node, timeouts, std::move(on_done));
  // Prebuilt (the reference appends the pod name; the caller only tests
  // is_wait(), so the message is not built per waiting gang member).
  static const Status kWait(Code::Wait, "one or more plugins asked to wait and no plugin rejected the pod");
  return kWait;
}

Status Framework::run_pre_bind(CycleState& s, const PodPtr& p, const std::string& node) {
  auto it = chain_.find(kPreBind);
  if (it == chain_.end()) return {};
  for (const auto& pl : it->second) {
    Status st = pl->pre_bind(s, p, node);
    if (!st.is_success()) return Status(Code::Error, "running PreBind plugin " + pl->name() + ": " + st.message());
  }
  return {};
}

Status Framework::run_bind(CycleState& s, const PodPtr& p, const std::string& node) {
  auto it = chain_.find(kBind);
  if (it == chain_.end()) return Status(Code::Skip);
  for (const auto& pl : it->second) {
    Status st = pl->bind(s, p, node);
    if (st.is_skip()) continue;
    if (!st.is_success()) return Status(Code::Error, "plugin \"" + pl->name() + "\" failed to bind pod: " + st.message());
    return st;
  }
  return Status(Code::Skip);
}

void Framework::run_post_bind(CycleState& s, const PodPtr& p, const std::string& node) {
  auto it = chain_.find(kPostBind);
  if (it == chain_.end()) return;
  for (const auto& pl : it->second) pl->post_bind(s, p, node);
}

std::vector<ClusterEvent> Framework::events_for(const std::string& plugin) const {
  auto it = by_name_.find(plugin);
  if (it == by_name_.end()) return {};
  return it->second->events_to_register();
}

std::vector<std::string> Framework::watched_kinds() const {
  std::vector<std::string> out;
  for (const auto& p : all_)
    for (const auto& k : p->watched_kinds())
      if (std::find(out.begin(), out.end(), k) == out.end()) out.push_back(k);
  return out;
}

void Framework::notify_capacity_freed() {
  for (const auto& p : capacity_watchers_) p->capacity_freed();
}

void Framework::dispatch_object_event(const std::string& kind, int type, const JsonPtr& obj, const JsonPtr& old) {
  auto it = kind_watchers_.find(kind);
  if (it == kind_watchers_.end()) return;
  for (const auto& p : it->second) p->on_object_event(kind, type, obj, old);
}

void Framework::start() {
  for (const auto& p : all_) p->start();
}

void Framework::stop() {
  for (const auto& p : all_) p->stop();
}

}  // namespace xsched
