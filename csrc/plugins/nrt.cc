// NodeResourceTopologyMatch with MI355X xGMI-aware gang placement.
//
// Reference: pkg/noderesourcetopology/{plugin.go,filter.go,score.go,
// least_allocated.go,most_allocated.go,balanced_allocation.go,
// pluginhelpers.go}:
//  * zones of type "Node" named node-<id> (0..63) form the NUMA list;
//  * Filter skips BestEffort pods and nodes without an NRT, and runs the
//    SingleNUMANode{Container,Pod}Level handlers: per resource a bitmask of
//    NUMA nodes that fit, AND-ed; non-Guaranteed pods always fit cpu/memory/
//    hugepages; non-native resources without NUMA affinity pass; container
//    scope subtracts the chosen (lowest) NUMA before the next container;
//  * Score: non-Guaranteed pods get 100; otherwise the minimum non-zero
//    per-NUMA strategy score (Least/Most/Balanced), mean over containers in
//    container scope.
//
// MI355X additions:
//  * GPU resources of a zone (amd.com/gpu, -xcd, -memory) are capped by the
//    scheduler's own GPU ledger for that socket, so zone availability is live
//    between exporter refreshes (the reference trusts the CR only);
//  * scoringStrategy XGMIGangAffinity: for a pod of a PodGroup, prefer the
//    node where the remaining ranks of the gang fit together (all RCCL hops on
//    the 7-link-per-GPU xGMI mesh of one 8x MI355X node), tightest fit first,
//    nodes already hosting siblings highest. Inside a node the xGMI mesh is
//    uniform, so there is no hop distance to optimise — only co-location.
//  * The sparse-NUMA-id index panic (Appendix C7) cannot happen: no array is
//    indexed by NUMA id.
#include <algorithm>
#include <cmath>
#include <map>

#include "common/log.h"
#include "framework/plugin.h"
#include "scheduler/cache.h"
#include "scheduler/gang_placement.h"
#include "scheduler/informers.h"

namespace xsched {
namespace {

using NumaNode = NumaZone;

// Per-cycle gang facts for XGMIGangAffinity, computed once in PreScore.
struct GangCtx : StateData {
  bool gang = false;
  uint64_t key = 0;         // Pod::pg_key of the gang
  int64_t remaining = 0;    // members still to place (>= 1)
  enum { kWhole, kXcd } kind = kWhole;
  int64_t amount = 0;       // per member: GPUs or XCDs
  // Snapshot nodes hosting members already (from the cache's group index):
  // the co-location test then reads only those NodeInfos, not every node's.
  std::vector<const NodeInfo*> hosts;
  bool hosts_known = false;
  std::shared_ptr<StateData> clone() const override { return std::make_shared<GangCtx>(*this); }
};
constexpr const char* kGangKey = "NodeResourceTopologyMatch/gang";

enum class Strategy { Least, Most, Balanced, XGMI };

int64_t value_units(int id, int64_t v) {  // Quantity.Value() semantics (cpu rounds up to cores)
  if (id == kCPU) return v >= 0 ? (v + 999) / 1000 : v / 1000;
  return v;
}

class TopologyMatch : public Plugin {
 public:
  // Zones come from the node's NRT and GPU ledger. XGMIGangAffinity scores a
  // gang member against the group's remaining ranks (cluster-wide), so it is
  // node-local only for pods outside a PodGroup.
  bool filter_node_local(const Pod&, const Snapshot&) const override { return true; }
  bool score_node_local(const Pod& p, const Snapshot&) const override {
    return strategy_ != Strategy::XGMI || p.pod_group.empty();
  }
  TopologyMatch(const Json& args, Handle& h)
      : Plugin("NodeResourceTopologyMatch", kPreFilter | kFilter | kPreScore | kScore), h_(h) {
    const Json& ss = args["scoringStrategy"];
    std::string t = ss["type"].str_or("LeastAllocated");
    if (t == "MostAllocated") strategy_ = Strategy::Most;
    else if (t == "BalancedAllocation") strategy_ = Strategy::Balanced;
    else if (t == "XGMIGangAffinity") strategy_ = Strategy::XGMI;
    else if (t == "LeastAllocated") strategy_ = Strategy::Least;
    else throw std::runtime_error("illegal scoring strategy found");
    for (const auto& r : ss["resources"].items()) weights_[res_id(r["name"].as_string())] = r["weight"].as_int(1);
    // xGMI gang co-location (gang_placement.h): on by default with the
    // XGMIGangAffinity strategy, in PreFilter when the profile enables it.
    colocation_ = GangPlacement::parse_mode(
        args["gangColocation"].str_or(strategy_ == Strategy::XGMI ? "Preferred" : "None"));
    if (h_.gangs) h_.gangs->set_mode(colocation_);
  }

  // ---- PreFilter: the gang's node set (the reference's alignment Filter,
  // filter.go:84-150,190-216, lifted from one NUMA zone to one xGMI mesh).
  Status pre_filter(CycleState& s, const Pod& p) override {
    if (colocation_ == GangPlacement::Mode::Off || !h_.gangs || !h_.snapshot || p.pod_group.empty() ||
        !GangPlacement::gang_demand(p.gpu_demand))
      return {};
    auto pg = h_.informers->pod_group_of(p);
    if (!pg || pg->min_member <= 1) return {};
    GangPlacement::Plan plan = h_.gangs->plan(*h_.snapshot, p, pg->min_member);
    if (!plan.gang) return {};
    if (!plan.started && h_.gang_planned) h_.gang_planned(p, plan.hostable);
    if (!plan.restriction) return {};
    plan.restriction->excluded = excluded_status();
    if (plan.restriction->list.empty() && plan.restriction->mask.empty() && !plan.restriction->fallback) {
      static const Status unhostable = [this] {
        Status x = Status::immortal(Code::Unschedulable,
                                    "no node can host every remaining rank of the PodGroup on one xGMI mesh "
                                    "(gangColocation: Required)");
        x.with_plugin(name_ptr());
        return x;
      }();
      return unhostable;
    }
    s.write(kNodeRestrictionKey, std::move(plan.restriction));
    return {};
  }
  const Status& excluded_status() const {
    static const Status st = [this] {
      Status x = Status::immortal(Code::Unschedulable,
                                  "node(s) cannot host the PodGroup's remaining ranks on one xGMI mesh");
      x.with_plugin(name_ptr());
      return x;
    }();
    return st;
  }

  int64_t weight(int id) const {
    auto it = weights_.find(id);
    return it == weights_.end() || it->second < 1 ? 1 : it->second;
  }

  std::vector<NumaNode> numa_list(const NodeResourceTopology& nrt, const NodeInfo& ni) const {
    std::vector<NumaNode> out = nrt.numa;  // precomputed at parse time
    const GpuNames& gn = *h_.gpu_names;
    int gid = gn.gpu_id(), xid = gn.xcd_id(), mid = gn.memory_id();
    const GpuLedger& L = ni.gpu;
    for (auto& n : out) {
      // Live GPU availability from the ledger for GPUs on this socket.
      if (n.id < 0 || n.id >= GpuLedger::kMaxZones || L.zone_gpus[n.id] == 0) continue;
      int64_t free_g = L.zone_whole[n.id], free_x = L.zone_xcds[n.id], free_m = L.zone_mem[n.id];
      if (int64_t* v = n.find(gid)) *v = std::min<int64_t>(*v, free_g);
      if (int64_t* v = n.find(xid)) *v = std::min<int64_t>(*v, free_x);
      if (int64_t* v = n.find(mid)) *v = std::min<int64_t>(*v, free_m);
    }
    return out;
  }

  static bool numa_suitable(QoS qos, int id, int64_t want, int64_t have) {
    if (qos != QoS::Guaranteed) {
      if (id == kCPU || id == kMemory || ResourceRegistry::get().is_hugepages(id)) return true;
    }
    return have >= want;
  }

  // Returns the lowest fitting NUMA id or -1.
  static int any_numa_fits(const std::vector<NumaNode>& nodes, const Res& req, QoS qos, const NodeInfo& ni) {
    uint64_t mask = ~uint64_t{0};
    for (uint64_t m = req.mask; m; m &= m - 1) {
      int id = __builtin_ctzll(m);
      int64_t want = req.v[id];
      if (want == 0) continue;
      if (!ni.allocatable.has(id)) return -1;
      bool affinity = false;
      uint64_t rmask = 0;
      for (const auto& n : nodes) {
        const int64_t* have = n.find(id);
        if (!have) continue;
        affinity = true;
        if (numa_suitable(qos, id, want, *have)) rmask |= uint64_t{1} << n.id;
      }
      if (!affinity && !ResourceRegistry::get().is_native(id)) continue;
      mask &= rmask;
      if (!mask) return -1;
    }
    // A mask with no NUMA constraint at all still has to name a zone.
    for (const auto& n : nodes)
      if (mask & (uint64_t{1} << n.id)) return n.id;
    return nodes.empty() ? -1 : -1;
  }

  // Live per-zone GPU availability, computed without allocation.
  struct LiveGpu {
    int64_t g[64], x[64], m[64];
    bool any[64];
  };
  static void live_gpu(const NodeInfo& ni, const NodeResourceTopology& nrt, LiveGpu& out) {
    const GpuLedger& L = ni.gpu;
    for (size_t z = 0; z < nrt.numa.size(); ++z) {
      int id = nrt.numa[z].id;
      bool ok = id >= 0 && id < GpuLedger::kMaxZones;
      out.any[z] = ok && L.zone_gpus[id] > 0;
      out.g[z] = out.any[z] ? L.zone_whole[id] : 0;
      out.x[z] = out.any[z] ? L.zone_xcds[id] : 0;
      out.m[z] = out.any[z] ? L.zone_mem[id] : 0;
    }
  }

  // Allocation-free resourcesAvailableInAnyNUMANodes for one request vector.
  bool fits_fast(const NodeResourceTopology& nrt, const NodeInfo& ni, const Res& req, QoS qos) const {
    if (nrt.numa.size() > 64) return true;
    const GpuNames& gn = *h_.gpu_names;
    int gid = gn.gpu_id(), xid = gn.xcd_id(), mid = gn.memory_id();
    LiveGpu live;
    bool live_ready = false;
    uint64_t mask = ~uint64_t{0};
    for (uint64_t m = req.mask; m; m &= m - 1) {
      int id = __builtin_ctzll(m);
      int64_t want = req.v[id];
      if (want == 0) continue;
      if (!ni.allocatable.has(id)) return false;
      bool affinity = false;
      uint64_t rmask = 0;
      for (size_t z = 0; z < nrt.numa.size(); ++z) {
        const int64_t* have = nrt.numa[z].find(id);
        if (!have) continue;
        affinity = true;
        int64_t h = *have;
        if (id == gid || id == xid || id == mid) {
          if (!live_ready) {
            live_gpu(ni, nrt, live);
            live_ready = true;
          }
          if (live.any[z]) h = std::min(h, id == gid ? live.g[z] : id == xid ? live.x[z] : live.m[z]);
        }
        if (numa_suitable(qos, id, want, h)) rmask |= uint64_t{1} << nrt.numa[z].id;
      }
      if (!affinity && !ResourceRegistry::get().is_native(id)) continue;
      mask &= rmask;
      if (!mask) return false;
    }
    for (const auto& z : nrt.numa)
      if (mask & (uint64_t{1} << z.id)) return true;
    return false;
  }

  Status filter(CycleState&, const Pod& p, const NodeInfo& ni) override {
    Status st = filter_impl(p, ni);
    if (XS_V(6)) log_filter(p, ni, st);
    return st;
  }

  // V(6): the node's NUMA zones with live GPU availability and the verdict
  // (the reference logs the same at V(6), pkg/noderesourcetopology/filter.go).
  void log_filter(const Pod& p, const NodeInfo& ni, const Status& st) const {
    if (ni.nrt) {
      const auto& reg = ResourceRegistry::get();
      for (const auto& n : numa_list(*ni.nrt, ni)) {
        Json avail = Json::object();
        for (const auto& [id, v] : n.res) avail.set(reg.name(id), Json(v));
        XS_LOGV(6, "numa zone").kv("node", ni.name()).kv("numa", n.id).kv("available", std::move(avail));
      }
    }
    XS_LOGV(6, "topology filter").kv("pod", p.key()).kv("node", ni.name()).kv("fits", st.is_success())
        .kv("reason", st.is_success() ? std::string() : st.message());
  }

  Status filter_impl(const Pod& p, const NodeInfo& ni) const {
    if (!ni.node) return Status::error("node not found");
    if (p.qos == QoS::BestEffort) return {};
    const NodeResourceTopology* nrt = ni.nrt.get();
    if (!nrt) return {};
    for (const auto& pol : nrt->topology_policies) {
      bool container_scope = pol == "SingleNUMANodeContainerLevel";
      if (container_scope && p.init_containers.empty() && p.containers.size() == 1) {
        // One container: container scope == pod scope, no subtraction needed.
        if (!fits_fast(*nrt, ni, p.containers[0].requests, p.qos))
          return Status::unschedulable("cannot align container: " + p.containers[0].name);
        continue;
      }
      if (pol == "SingleNUMANodePodLevel") {
        if (!fits_fast(*nrt, ni, p.request(), p.qos)) {
          thread_local std::string memo_uid;
          thread_local Status memo;
          if (memo_uid != p.uid()) {
            memo = Status::unschedulable("cannot align pod: " + p.name());
            memo_uid = p.uid();
          }
          return memo;
        }
        continue;
      }
      if (container_scope) {
        auto nodes = numa_list(*nrt, ni);
        for (const auto& c : p.init_containers)
          if (any_numa_fits(nodes, c.requests, p.qos, ni) < 0)
            return Status::unschedulable("cannot align init container: " + c.name);
        for (const auto& c : p.containers) {
          int id = any_numa_fits(nodes, c.requests, p.qos, ni);
          if (id < 0) return Status::unschedulable("cannot align container: " + c.name);
          for (auto& n : nodes)
            if (n.id == id)
              for (uint64_t m = c.requests.mask; m; m &= m - 1) {
                int r = __builtin_ctzll(m);
                if (int64_t* v = n.find(r)) *v -= c.requests.v[r];
              }
        }
      }
    }
    return {};
  }

  int64_t strategy_score(const Res& req, const NumaNode& n) const {
    if (strategy_ == Strategy::Balanced) {
      double fr[kMaxRes];
      int k = 0;
      for (uint64_t m = req.mask; m; m &= m - 1) {
        int id = __builtin_ctzll(m);
        const int64_t* have = n.find(id);
        int64_t cap = have ? value_units(id, *have) : 0;
        double f = cap == 0 ? 1.0 : static_cast<double>(value_units(id, req.v[id])) / static_cast<double>(cap);
        if (f > 1) return 0;
        fr[k++] = f;
      }
      if (k < 2) return kMaxNodeScore;  // gonum Variance of <2 samples is 0
      double mean = 0;
      for (int i = 0; i < k; ++i) mean += fr[i];
      mean /= k;
      double var = 0;
      for (int i = 0; i < k; ++i) var += (fr[i] - mean) * (fr[i] - mean);
      var /= (k - 1);  // stat.Variance is the unbiased estimator
      return static_cast<int64_t>((1 - var) * kMaxNodeScore);
    }
    int64_t num = 0, wsum = 0;
    for (uint64_t m = req.mask; m; m &= m - 1) {
      int id = __builtin_ctzll(m);
      const int64_t* have = n.find(id);
      int64_t cap = have ? value_units(id, *have) : 0;
      int64_t want = value_units(id, req.v[id]);
      int64_t s = 0;
      if (cap != 0 && want <= cap)
        s = strategy_ == Strategy::Most ? want * kMaxNodeScore / cap : (cap - want) * kMaxNodeScore / cap;
      num += s * weight(id);
      wsum += weight(id);
    }
    return wsum ? num / wsum : 0;
  }

  int64_t min_numa_score(const Res& req, const std::vector<NumaNode>& nodes) const {
    int64_t mn = 0;
    for (const auto& n : nodes) {
      int64_t s = strategy_score(req, n);
      if (mn == 0 || (s != 0 && s < mn)) mn = s;
    }
    return mn;
  }

  // PreScore: gang facts shared by every node's Score (one PodGroup lookup
  // and one assigned-count read per cycle instead of per node).
  Status pre_score(CycleState& s, const Pod& p, const NodeList&) override {
    if (strategy_ != Strategy::XGMI) return {};
    auto ctx = std::make_shared<GangCtx>();
    if (!p.pod_group.empty()) {
      auto pg = h_.informers->pod_group_of(p);
      const GpuDemand& d = p.gpu_demand;
      if (pg && pg->min_member > 1 && d.amount > 0 && (d.kind == GpuDemand::Gpu || d.kind == GpuDemand::Xcd)) {
        ctx->gang = true;
        ctx->key = p.pg_key;
        ctx->remaining = std::max<int64_t>(1, pg->min_member - h_.cache->assigned_in_group(ctx->key));
        ctx->kind = d.kind == GpuDemand::Gpu ? GangCtx::kWhole : GangCtx::kXcd;
        ctx->amount = d.amount;
        if (h_.snapshot) {
          for (const auto& node : h_.cache->nodes_of_group(ctx->key))
            if (auto ni = h_.snapshot->get(node)) ctx->hosts.push_back(ni.get());
          ctx->hosts_known = true;
        }
      }
    }
    s.write(kGangKey, ctx);
    return {};
  }

  static bool co_located(const GangCtx& c, const NodeInfo& ni) {
    if (!c.hosts_known) return ni.pg_pods(c.key) > 0;
    for (const NodeInfo* h : c.hosts)
      if (h == &ni) return ni.pg_pods(c.key) > 0;
    return false;
  }
  static int64_t fit_score(int64_t remaining, int64_t free, bool co) {
    if (free <= 0) return 0;
    bool fits_all = remaining <= free;
    if (fits_all && co) return 100;
    if (fits_all) return 60 + 30 * remaining / free;  // tightest whole-gang fit first
    if (co) return 50;
    return 40 * std::min(free, remaining) / remaining;  // most of the gang on one node
  }
  // fit_score for one gang demand over a cycle's nodes: the few distinct
  // (free, co-located) pairs are computed once each (no division per node).
  struct FitMemo {
    int64_t remaining = -1;
    int64_t v[2][65];
    int64_t get(int64_t r, int64_t free, bool co) {
      if (free < 0 || free > 64) return fit_score(r, free, co);
      if (r != remaining) {
        remaining = r;
        std::fill(&v[0][0], &v[0][0] + 2 * 65, int64_t{-1});
      }
      int64_t& slot = v[co][free];
      if (slot < 0) slot = fit_score(r, free, co);
      return slot;
    }
  };
  // gang_score for a whole-GPU rank given the node's free GPUs.
  static int64_t whole_gang_score(const GangCtx& c, int64_t free_gpus, const NodeInfo& ni) {
    if (free_gpus <= 0) return 0;
    return fit_score(c.remaining * c.amount, free_gpus, co_located(c, ni));
  }
  // Gang co-location score in [0, 100] (XGMIGangAffinity).
  static int64_t gang_score(const GangCtx& c, const NodeInfo& ni) {
    if (!c.gang) return 50;
    const GpuLedger& L = ni.gpu;
    int64_t per = 0, free = 0;
    if (c.kind == GangCtx::kWhole) {
      per = c.amount;
      free = L.free_gpus();
    } else {
      // A member consumes whole partitions: on SPX GPUs a 2-XCD rank burns 8.
      for (int g = 0; g < L.gpu_count; ++g) {
        if (L.monopoly[g] > 0 || L.xcds_per_part(g) <= 0) continue;
        int64_t xpp = L.xcds_per_part(g);
        int64_t use = (c.amount + xpp - 1) / xpp * xpp;
        if (per == 0 || use < per) per = use;
      }
      if (per == 0) return 0;
      free = L.free_xcds();
    }
    if (free <= 0) return 0;
    return fit_score(c.remaining * per, free, co_located(c, ni));
  }

  std::pair<int64_t, Status> score(CycleState& s, const Pod& p, const NodeInfo& ni) override {
    if (strategy_ == Strategy::XGMI) {
      if (auto* c = s.read_as<GangCtx>(kGangKey)) return {gang_score(*c, ni), {}};
      // PreScore not enabled for this profile: derive the context per node.
      CycleState local;
      NodeList none;
      pre_score(local, p, none);
      return {gang_score(*local.read_as<GangCtx>(kGangKey), ni), {}};
    }
    if (p.qos != QoS::Guaranteed) return {kMaxNodeScore, {}};
    NRTPtr nrt = ni.nrt;
    if (!nrt) return {0, {}};
    for (const auto& pol : nrt->topology_policies) {
      if (pol != "SingleNUMANodePodLevel" && pol != "SingleNUMANodeContainerLevel") continue;
      auto nodes = numa_list(*nrt, ni);
      if (pol == "SingleNUMANodePodLevel") return {min_numa_score(p.request(), nodes), {}};
      double sum = 0;
      size_t n = 0;
      for (const auto& c : p.init_containers) {
        sum += static_cast<double>(min_numa_score(c.requests, nodes));
        ++n;
      }
      for (const auto& c : p.containers) {
        sum += static_cast<double>(min_numa_score(c.requests, nodes));
        ++n;
      }
      return {n ? static_cast<int64_t>(sum / static_cast<double>(n)) : 0, {}};
    }
    return {0, {}};
  }

  // XGMIGangAffinity over many nodes: the gang context is read once.
  Status score_many(CycleState& s, const Pod& p, const NodeList& nodes, const char* skip,
                    std::vector<NodeScore>& out, const int* pos) override {
    const GangCtx* c = strategy_ == Strategy::XGMI ? s.read_as<GangCtx>(kGangKey) : nullptr;
    if (!c) return Plugin::score_many(s, p, nodes, skip, out, pos);
    const Snapshot* snap = h_.snapshot;
    if (pos && snap && c->gang && c->kind == GangCtx::kWhole && snap->free_whole.size() == snap->nodes.size()) {
      // Whole-GPU ranks: free GPUs from the snapshot's contiguous array; only
      // the few nodes already hosting the gang are dereferenced.
      FitMemo fm;
      const int64_t r = c->remaining * c->amount;
      for (size_t i = 0; i < nodes.size(); ++i) {
        if (skip && skip[i]) continue;
        const int64_t free = snap->free_whole[pos[i]];
        out[i].score = free <= 0 ? 0 : fm.get(r, free, co_located(*c, *nodes[i]));
      }
      return {};
    }
    if (pos && snap && c->gang && c->kind == GangCtx::kXcd && snap->part_mask.size() == snap->nodes.size()) {
      // XCD ranks: a member's partition footprint depends only on which
      // partition sizes the node offers (Snapshot::part_mask), so it is
      // tabulated once per cycle; free XCDs come from the contiguous array.
      int64_t per_of[16];
      for (int m = 0; m < 16; ++m) {
        int64_t per = 0;
        for (int b = 0; b < 4; ++b) {
          if (!(m & (1 << b))) continue;
          const int64_t xpp = 1 << b;
          const int64_t use = (c->amount + xpp - 1) / xpp * xpp;
          if (per == 0 || use < per) per = use;
        }
        per_of[m] = per;
      }
      // One memo per partition mask: its gang demand (remaining x per) is
      // fixed for the call, so nodes of mixed masks do not refill a shared
      // memo back and forth (that refill was a third of this loop's time at
      // 1,024 nodes, profiles/r5ad_samples_n1024.txt).
      FitMemo fm[16];
      for (size_t i = 0; i < nodes.size(); ++i) {
        if (skip && skip[i]) continue;
        const uint8_t m = snap->part_mask[pos[i]] & 15;
        const int64_t per = per_of[m];
        const int64_t free = snap->free_xcd[pos[i]];
        out[i].score = per == 0 || free <= 0 ? 0 : fm[m].get(c->remaining * per, free, co_located(*c, *nodes[i]));
      }
      return {};
    }
    for (size_t i = 0; i < nodes.size(); ++i)
      if (!skip || !skip[i]) out[i].score = gang_score(*c, *nodes[i]);
    return {};
  }

  std::vector<ClusterEvent> events_to_register() const override {
    return {{"Pod", kDelete, ""}, {"Node", kAdd | kUpdateNodeAllocatable, ""}, {"NodeResourceTopology", kAdd | kUpdate, ""}};
  }

  // Unit-test hook: "gangPlan" returns the co-location plan PreFilter would
  // use for p (allowed node names, fallback, hostable, remaining ranks).
  Json debug_call(const std::string& what, CycleState& s, const PodPtr& p, const Json& args) override {
    if (what != "gangPlan") return Plugin::debug_call(what, s, p, args);
    Json out = Json::object();
    out.set("mode", Json(GangPlacement::mode_name(colocation_)));
    auto pg = p->pod_group.empty() ? nullptr : h_.informers->pod_group_of(*p);
    if (!pg || !h_.gangs || !h_.snapshot) {
      out.set("gang", Json(false));
      return out;
    }
    GangPlacement::Plan plan = h_.gangs->plan(*h_.snapshot, *p, pg->min_member);
    out.set("gang", Json(plan.gang));
    out.set("started", Json(plan.started));
    out.set("remaining", Json(plan.remaining));
    out.set("hostable", Json(plan.hostable));
    out.set("restricted", Json(static_cast<bool>(plan.restriction)));
    if (plan.restriction) {
      Json nodes = Json::array();
      const auto& r = *plan.restriction;
      for (size_t i = 0; i < h_.snapshot->names.size(); ++i)
        if ((!r.mask.empty() || !r.list.empty()) && r.allows(static_cast<int>(i)))
          nodes.push_back(Json(h_.snapshot->names[i]));
      out.set("nodes", std::move(nodes));
      out.set("fallback", Json(r.fallback));
    }
    out.set("openGangs", Json(static_cast<int64_t>(h_.gangs->open_gangs())));
    return out;
  }

 private:
  Handle& h_;
  Strategy strategy_ = Strategy::Least;
  GangPlacement::Mode colocation_ = GangPlacement::Mode::Off;
  std::map<int, int64_t> weights_;
};

PluginRegistrar reg("NodeResourceTopologyMatch",
                    [](const Json& a, Handle& h) { return std::make_shared<TopologyMatch>(a, h); });

}  // namespace

void link_nrt_plugin() {}

}  // namespace xsched
