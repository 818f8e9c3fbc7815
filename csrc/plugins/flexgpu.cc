// FlexGPU for AMD Instinct MI355X: whole-GPU, compute-partition (XCD) and
// shared-HBM-slice bin-packing.
//
// Reference behaviour: pkg/flexgpu/flex_gpu.go:41-242 and gpu_node.go:30-199
// (Filter/Score/NormalizeScore(reverse)/Reserve/Unreserve/Bind, index
// annotation copied onto the pod by the Binding). MI355X model (SURVEY.md
// Appendix D, decided here):
//
//   amd.com/gpu         k whole physical GPUs (exclusive)       -> "amd.com/gpu-index": "0,3"
//   amd.com/gpu-xcd     x XCDs of compute partitions (CPX/QPX/  -> "amd.com/gpu-index": "2",
//                       DPX), exclusive, on one GPU                 "amd.com/gpu-partitions": "2:4,2:5"
//   amd.com/gpu-memory  a slice of one partition's HBM, shared  -> "amd.com/gpu-index": "1",
//                       (time-sliced), best-fit packed             "amd.com/gpu-partitions": "1:0"
//
// A pod requests exactly one kind (more is UnschedulableAndUnresolvable, as
// gpu+memory is in flex_gpu.go:58-61); demand is the sum of container LIMITS.
// The node's compute-partition mode comes from the node agent (label
// amd.com/gpu.compute-partition or the amd.com/gpu-topology annotation) and
// is node state: the scheduler never repartitions. Per-partition HBM =
// per-GPU memory / partitions (per-GPU memory = allocatable memory / GPUs,
// the reference's homogeneous split, gpu_node.go:51-55).
//
// Deliberate fixes of reference quirks:
//  C1 value semantics + a real best-fit order for memory slices;
//  C2 GPU indexes are bounds-checked (bad annotations are ignored, no panic);
//  C3 whole-GPU pods are checked per GPU in Filter (Reserve can no longer
//     fail after Filter passed) and k > 1 GPUs are supported.
#include <algorithm>
#include <cstdint>
#include <string>

#include "common/log.h"
#include "framework/plugin.h"
#include "scheduler/cache.h"

namespace xsched {
namespace {

constexpr const char* kFlexGPUStateKey = "FlexGPU/assignment";

using Demand = GpuDemand;

struct Placement {
  std::vector<int> gpus;
  std::vector<std::pair<int, int>> parts;
  bool ok() const { return !gpus.empty(); }
};

// k untouched GPUs; NUMA-local when possible (the NUMA node with the fewest
// free GPUs that still fits, i.e. bin-pack sockets), lowest indexes first.
Placement place_whole(const GpuLedger& L, int64_t k) {
  Placement pl;
  if (k <= 0) k = 1;
  // Free GPUs per NUMA node, counted in place (no per-call containers: this
  // runs in every whole-GPU pod's Reserve).
  int n_free = 0;
  for (int g = 0; g < L.gpu_count; ++g) n_free += L.whole_gpu_free(g);
  if (n_free < k) return pl;
  // The NUMA node with the fewest free GPUs that still fits (lowest id among
  // equals); -1 ("unknown") never qualifies. Used only when the free GPUs
  // span more than one NUMA value or sit on one known node.
  int best_numa = INT32_MIN, best_count = 0, distinct = 0, first_numa = INT32_MAX;
  for (int g = 0; g < L.gpu_count; ++g) {
    if (!L.whole_gpu_free(g)) continue;
    const int numa = L.numa[g];
    bool seen = false;
    for (int h = 0; h < g && !seen; ++h) seen = L.whole_gpu_free(h) && L.numa[h] == numa;
    if (seen) continue;  // counted with its first GPU
    ++distinct;
    first_numa = std::min(first_numa, numa);
    if (numa < 0) continue;
    int count = 0;
    for (int h = g; h < L.gpu_count; ++h) count += L.whole_gpu_free(h) && L.numa[h] == numa;
    if (count < k) continue;
    if (best_numa == INT32_MIN || count < best_count || (count == best_count && numa < best_numa)) {
      best_numa = numa;
      best_count = count;
    }
  }
  const bool by_numa = distinct > 1 || (distinct == 1 && first_numa >= 0);
  for (int g = 0; g < L.gpu_count && static_cast<int64_t>(pl.gpus.size()) < k; ++g)
    if (L.whole_gpu_free(g) && (!by_numa || best_numa == INT32_MIN || L.numa[g] == best_numa)) pl.gpus.push_back(g);
  return pl;
}

// x XCDs from exclusive partitions of one GPU. The GPU is chosen by
// (wasted XCDs, free XCDs): a 2-XCD request on a CPX GPU wastes nothing, on
// an SPX GPU it strands 6 XCDs, so partitioned GPUs win whenever they fit;
// among equals the fullest GPU (best fit). Lowest free partitions inside it.
int xcd_waste(const GpuLedger& L, int g, int64_t x) {
  int xpp = L.xcds_per_part(g);
  int need = static_cast<int>((x + xpp - 1) / xpp);
  return static_cast<int>(need * xpp - x);
}

// `build` false: only *waste_out is wanted (Score), no placement vectors.
Placement place_xcd(const GpuLedger& L, int64_t x, int* waste_out = nullptr, bool build = true) {
  Placement pl;
  if (x <= 0) return pl;
  int best_g = -1, best_free = 1 << 30, best_waste = 1 << 30;
  for (int g = 0; g < L.gpu_count; ++g) {
    if (L.monopoly[g] > 0) continue;
    int xpp = L.xcds_per_part(g);
    if (xpp <= 0) continue;
    int need = static_cast<int>((x + xpp - 1) / xpp);
    int free = L.free[g].free_slots;
    if (free < need) continue;
    int free_x = free * xpp;
    int waste = xcd_waste(L, g, x);
    if (waste < best_waste || (waste == best_waste && free_x < best_free)) {
      best_waste = waste;
      best_free = free_x;
      best_g = g;
    }
  }
  if (waste_out) *waste_out = best_g < 0 ? 0 : best_waste;
  if (best_g < 0 || !build) return pl;
  int xpp = L.xcds_per_part(best_g);
  int need = static_cast<int>((x + xpp - 1) / xpp);
  for (int p = 0; p < L.parts[best_g] && static_cast<int>(pl.parts.size()) < need; ++p)
    if (L.slot_free(best_g, p)) pl.parts.emplace_back(best_g, p);
  pl.gpus.push_back(best_g);
  return pl;
}

// Memory slice on the partition with the least remaining memory after
// placement (best fit, value semantics — fixes Appendix C1). A slice never
// breaks an untouched SPX GPU while any other partition can take it: that GPU
// is the only kind a whole-GPU (training-rank) pod can use.
// `build` false: only *breaks_whole is wanted (Score), no placement vectors.
Placement place_memory(const GpuLedger& L, int64_t m, bool* breaks_whole = nullptr, bool build = true) {
  Placement pl;
  int bg = -1, bp = -1;
  int64_t best_remain = 0;
  bool best_breaks = true;
  for (int g = 0; g < L.gpu_count; ++g) {
    // No partition of g has m free (the ledger's per-GPU maximum): skip its
    // partitions (-1 for a monopolised GPU).
    if (L.monopoly[g] > 0 || L.free[g].max_slot_mem < m) continue;
    int64_t cap = L.part_mem(g);
    bool breaks = L.whole_gpu_free(g);
    for (int p = 0; p < L.parts[g]; ++p) {
      const auto& s = L.slots[L.offset[g] + p];
      if (s.exclusive > 0) continue;
      int64_t remain = cap - s.used_mem - m;
      if (remain < 0) continue;
      if (bg < 0 || (!breaks && best_breaks) || (breaks == best_breaks && remain < best_remain)) {
        bg = g;
        bp = p;
        best_remain = remain;
        best_breaks = breaks;
      }
    }
  }
  if (breaks_whole) *breaks_whole = bg >= 0 && best_breaks;
  if (bg < 0 || !build) return pl;
  pl.gpus.push_back(bg);
  pl.parts.emplace_back(bg, bp);
  return pl;
}

Placement place(const GpuLedger& L, const Demand& d) {
  switch (d.kind) {
    case Demand::Gpu: return place_whole(L, d.amount);
    case Demand::Xcd: return place_xcd(L, d.amount);
    case Demand::Memory: return place_memory(L, d.amount);
    default: return {};
  }
}

std::string join_ints(const std::vector<int>& v) {
  std::string s;
  for (size_t i = 0; i < v.size(); ++i) s += (i ? "," : "") + std::to_string(v[i]);
  return s;
}

std::string join_parts(const std::vector<std::pair<int, int>>& v) {
  std::string s;
  for (size_t i = 0; i < v.size(); ++i) s += (i ? "," : "") + std::to_string(v[i].first) + ":" + std::to_string(v[i].second);
  return s;
}

// The placement Reserve chose, as the annotation values Bind writes; the
// Json object is built by Bind, on a binder thread, not in the scheduling
// cycle.
struct AssignmentState : StateData {
  std::string index, partitions;  // partitions: empty for whole-GPU / HBM pods
  Json annotations(const GpuNames& gn) const {
    Json a = Json::object();
    a.set(gn.index_annotation, Json(index));
    if (!partitions.empty()) a.set(gn.partition_annotation, Json(partitions));
    return a;
  }
  std::shared_ptr<StateData> clone() const override { return std::make_shared<AssignmentState>(*this); }
};

class FlexGPU : public Plugin {
 public:
  // Filter/Score read only the node's GPU ledger, allocatable and the pod's demand.
  bool filter_node_local(const Pod&, const Snapshot&) const override { return true; }
  bool score_node_local(const Pod&, const Snapshot&) const override { return true; }
  // Resource/annotation names come from the scheduler (GpuNames::from_args
  // of this plugin's args, checked equal across profiles in Scheduler()).
  FlexGPU(const Json&, Handle& h) : Plugin("FlexGPU", kFilter | kScore | kReserve | kBind), h_(h), gn_(*h.gpu_names) {}

  Status filter(CycleState&, const Pod& p, const NodeInfo& ni) override {
    const Demand& d = p.gpu_demand;
    if (XS_V(6)) log_filter(p, ni);
    if (d.kind == Demand::None) return {};
    if (d.kind == Demand::Conflict) return Status::unresolvable("pod conflict resources");
    const GpuNames& gn = gn_;
    int gid = gn.gpu_id();
    int kid = d.kind == Demand::Gpu ? gid : d.kind == Demand::Xcd ? gn.xcd_id() : gn.memory_id();
    if (!ni.allocatable.has(gid) || !ni.allocatable.has(kid)) return Status::unresolvable("unknown resource type");
    // Node-level sum check (flex_gpu.go:82-98).
    if (ni.requested.get(kid) + d.amount > ni.allocatable.get(kid)) return failure(kid, false);
    if (!fits(ni.gpu, d)) return failure(kid, true);
    return {};
  }

  // V(6) dump of the pod's limits and the node's GPU ledger, as the
  // reference's Filter does (pkg/flexgpu/flex_gpu.go:42-50,103-107).
  void log_filter(const Pod& p, const NodeInfo& ni) const {
    XS_LOGV(6, "pod info").kv("point", "filter").kv("pod", p.key()).kv("node", ni.name());
    for (const auto& c : p.containers)
      for (int id : {gn_.gpu_id(), gn_.xcd_id(), gn_.memory_id()})
        if (c.limits.has(id))
          XS_LOGV(6, "resource limit").kv("container", c.name).kv(ResourceRegistry::get().name(id), c.limits.get(id));
    const GpuLedger& L = ni.gpu;
    for (int g = 0; g < L.gpu_count; ++g) {
      const auto& f = L.free[g];
      XS_LOGV(6, "node gpu usages").kv("node", ni.name()).kv("gpu", g).kv("partitions", L.parts[g])
          .kv("wholeFree", f.whole).kv("freeSlots", f.free_slots).kv("freeXcds", f.xcds).kv("freeMemory", f.mem)
          .kv("numa", g < static_cast<int>(L.numa.size()) ? L.numa[g] : -1);
    }
  }

  // Prebuilt per resource id (Filter fails on most nodes of a busy cluster).
  static Status failure(int kid, bool no_fit) {
    thread_local std::unordered_map<int, std::pair<Status, Status>> memo;
    auto it = memo.find(kid);
    if (it == memo.end()) {
      const std::string n = ResourceRegistry::get().name(kid);
      it = memo.emplace(kid, std::make_pair(Status::interned(Code::Unschedulable, {"insufficient resource " + n}),
                                            Status::interned(Code::Unschedulable, {"no fit indexes resource " + n})))
               .first;
    }
    return no_fit ? it->second.second : it->second.first;
  }

  // Allocation-free feasibility check (Filter runs per node per pod; the
  // concrete placement is only materialized in Reserve).
  static bool fits(const GpuLedger& L, const Demand& d) {
    switch (d.kind) {
      case Demand::Gpu:
        return L.free_gpus() >= (d.amount > 0 ? d.amount : 1);
      case Demand::Xcd: {
        if (d.amount <= 0 || L.free_xcds() < d.amount) return false;
        for (int g = 0; g < L.gpu_count; ++g) {
          int xpp = L.xcds_per_part(g);
          if (xpp <= 0) continue;
          if (L.free[g].free_slots >= static_cast<int>((d.amount + xpp - 1) / xpp)) return true;
        }
        return false;
      }
      case Demand::Memory: {
        if (L.free_memory() < d.amount) return false;
        for (int g = 0; g < L.gpu_count; ++g)
          if (L.free[g].max_slot_mem >= d.amount) return true;
        return false;
      }
      default: return false;
    }
  }

  std::pair<int64_t, Status> score(CycleState&, const Pod& p, const NodeInfo& ni) override {
    const Demand& d = p.gpu_demand;
    switch (d.kind) {
      case Demand::Gpu: return {ni.gpu.free_gpus(), {}};
      case Demand::Xcd: {
        // Stranded XCDs dominate: a node that can host the slice without
        // waste always outranks one that would burn a whole SPX GPU on it.
        int waste = 0;
        place_xcd(ni.gpu, d.amount, &waste, /*build=*/false);
        return {ni.gpu.free_xcds() + 64 * waste, {}};
      }
      case Demand::Memory: {
        // Breaking a whole SPX GPU for a slice costs more than any packing gain.
        bool breaks = false;
        place_memory(ni.gpu, d.amount, &breaks, /*build=*/false);
        return {ni.gpu.free_memory() + (breaks ? 8 * ni.gpu.mem_per_gpu : 0), {}};
      }
      default: return {0, {}};
    }
  }
  bool has_normalize_score() const override { return true; }
  Status normalize_score(CycleState&, const Pod&, std::vector<NodeScore>& s) override {
    default_normalize_score(kMaxNodeScore, true, s);  // fewer free -> higher: node-level bin packing
    return {};
  }

  Status reserve(CycleState& s, const PodPtr& p, const std::string& node) override {
    const Demand& d = p->gpu_demand;
    if (d.kind == Demand::None) return {};
    if (d.kind == Demand::Conflict) return Status::unresolvable("pod conflict resources");
    NodeInfoPtr ni = h_.snapshot ? h_.snapshot->get(node) : nullptr;
    if (!ni) return Status::error("getting node \"" + node + "\" from Snapshot");
    Placement pl = place(ni->gpu, d);
    if (!pl.ok()) return Status::unschedulable("allocate index fail");
    XS_LOGV(6, "assigned gpu indexes").kv("pod", p->key()).kv("node", node).kv("indexes", join_ints(pl.gpus))
        .kv("partitions", join_parts(pl.parts));
    const GpuNames& gn = gn_;
    auto st = std::make_shared<AssignmentState>();
    st->index = join_ints(pl.gpus);
    if (!pl.parts.empty()) st->partitions = join_parts(pl.parts);
    h_.cache->annotate_assumed_pod(p->uid(), [&](Pod& cp) {
      StrMap& am = cp.meta.annotations.mut();
      auto put = [&](const std::string& k, const std::string& v) {
        for (auto& a : am)
          if (a.first == k) {
            a.second = v;
            return;
          }
        am.emplace_back(k, v);
      };
      put(gn.index_annotation, st->index);
      if (!st->partitions.empty()) put(gn.partition_annotation, st->partitions);
      cp.set_gpu_assignment(pl.gpus, pl.parts, gn);  // what the annotations just written parse to
    }, /*recompute=*/false);
    s.write(kFlexGPUStateKey, st);
    return {};
  }

  void unreserve(CycleState& s, const PodPtr& p, const std::string&) override {
    const GpuNames& gn = gn_;
    s.erase(kFlexGPUStateKey);
    if (!h_.cache->is_assumed(p->uid())) return;
    h_.cache->mutate_pod(p->uid(), [&](Pod& cp) {
      auto& a = cp.meta.annotations.mut();
      a.erase(std::remove_if(a.begin(), a.end(),
                             [&](const auto& kv) {
                               return kv.first == gn.index_annotation || kv.first == gn.partition_annotation;
                             }),
              a.end());
    });
  }

  Status bind(CycleState& s, const PodPtr& p, const std::string& node) override {
    Json ann = Json::object();
    if (auto* st = s.read_as<AssignmentState>(kFlexGPUStateKey)) ann = st->annotations(gn_);
    try {
      h_.client->bind(*p, node, ann);
    } catch (const std::exception& e) {
      return Status::error(e.what());
    }
    return {};
  }

  std::vector<ClusterEvent> events_to_register() const override {
    return {{"Pod", kDelete, ""}, {"Node", kAdd | kUpdateNodeAllocatable | kUpdateNodeLabel, ""}};
  }

 private:
  Handle& h_;
  const GpuNames& gn_;
};

PluginRegistrar reg("FlexGPU", [](const Json& a, Handle& h) { return std::make_shared<FlexGPU>(a, h); });

}  // namespace

void link_flexgpu_plugin() {}

}  // namespace xsched
