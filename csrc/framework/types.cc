#include "framework/types.h"

#include <algorithm>

namespace xsched {

const char* code_name(Code c) {
  switch (c) {
    case Code::Success: return "Success";
    case Code::Error: return "Error";
    case Code::Unschedulable: return "Unschedulable";
    case Code::UnschedulableAndUnresolvable: return "UnschedulableAndUnresolvable";
    case Code::Wait: return "Wait";
    case Code::Skip: return "Skip";
  }
  return "Unknown";
}

const std::vector<std::string>& Status::reasons() const {
  static const std::vector<std::string> kNone;
  return reasons_ ? *reasons_ : kNone;
}

const std::string& Status::intern_plugin(std::string_view p) { return IStr::intern(p); }

Status Status::interned(Code c, std::vector<std::string> reasons) {
  static std::mutex mu;
  static auto* table = new std::map<std::pair<int, std::vector<std::string>>, const std::vector<std::string>*>();
  std::lock_guard<std::mutex> g(mu);
  auto key = std::make_pair(static_cast<int>(c), std::move(reasons));
  auto it = table->find(key);
  if (it == table->end()) {
    auto* r = new std::vector<std::string>(key.second);  // never freed (bounded by distinct verdicts)
    it = table->emplace(std::move(key), r).first;
  }
  Status s(c);
  s.reasons_ = it->second;
  return s;
}

const std::string& Status::failed_plugin() const {
  static const std::string kNone;
  return plugin_ ? *plugin_ : kNone;
}

std::string Status::message() const {
  std::string s;
  if (!reasons_) return s;
  for (size_t i = 0; i < reasons_->size(); ++i) {
    if (i) s += ", ";
    s += (*reasons_)[i];
  }
  return s;
}

// ----------------------------------------------------------- CycleState ----
uint64_t CycleState::next_version() {
  static std::atomic<uint64_t> counter{1};
  return counter.fetch_add(1, std::memory_order_relaxed);
}

std::shared_ptr<StateData> CycleState::read(std::string_view key) const {
  std::shared_lock<std::shared_mutex> g(mu_);
  for (const auto& kv : kv_)
    if (*kv.first == key) return kv.second;
  return nullptr;
}

StateData* CycleState::read_raw(std::string_view key) const {
  std::shared_lock<std::shared_mutex> g(mu_);
  for (const auto& kv : kv_)
    if (*kv.first == key) return kv.second.get();
  return nullptr;
}

namespace {
// Plugins write a handful of constant keys every cycle: a per-thread list of
// the keys seen so far skips the intern table's lock and hash.
const std::string* intern_key(std::string_view key) {
  thread_local std::vector<const std::string*> seen;
  for (const std::string* k : seen)
    if (*k == key) return k;
  const std::string* k = &IStr::intern(key);
  if (seen.size() < 64) seen.push_back(k);
  return k;
}
}  // namespace

void CycleState::write(std::string_view key, std::shared_ptr<StateData> v) {
  std::unique_lock<std::shared_mutex> g(mu_);
  version_.store(next_version(), std::memory_order_release);
  for (auto& kv : kv_)
    if (*kv.first == key) {
      kv.second = std::move(v);
      return;
    }
  kv_.emplace_back(intern_key(key), std::move(v));
}

void CycleState::erase(std::string_view key) {
  std::unique_lock<std::shared_mutex> g(mu_);
  version_.store(next_version(), std::memory_order_release);
  kv_.erase(std::remove_if(kv_.begin(), kv_.end(), [&](const auto& kv) { return *kv.first == key; }), kv_.end());
}

std::shared_ptr<CycleState> CycleState::clone() const {
  auto c = std::make_shared<CycleState>();
  std::shared_lock<std::shared_mutex> g(mu_);
  for (const auto& kv : kv_) {
    if (!kv.second) continue;
    auto cl = kv.second->clone();
    c->kv_.emplace_back(kv.first, cl ? cl : kv.second);
  }
  c->record_metrics = record_metrics;
  c->nominated = nominated;
  c->filter_skip = filter_skip;
  return c;
}

// ------------------------------------------------------------ GpuLedger ----
void GpuLedger::init(const Node& n) {
  gpu_count = n.gpu_count;
  mem_per_gpu = n.gpu_memory_per_gpu;
  parts = n.gpu_partitions;
  numa = n.gpu_numa;
  parts.resize(gpu_count, 1);
  numa.resize(gpu_count, -1);
  offset.assign(gpu_count + 1, 0);
  for (int g = 0; g < gpu_count; ++g) offset[g + 1] = offset[g] + std::max(1, parts[g]);
  monopoly.assign(gpu_count, 0);
  slots.assign(offset[gpu_count], Slot{});
  free.assign(gpu_count, GpuFree{});
  tot_whole = tot_xcds = 0;
  tot_mem = 0;
  std::fill(std::begin(zone_gpus), std::end(zone_gpus), 0);
  std::fill(std::begin(zone_whole), std::end(zone_whole), 0);
  std::fill(std::begin(zone_xcds), std::end(zone_xcds), 0);
  std::fill(std::begin(zone_mem), std::end(zone_mem), 0);
  zone_n = 0;
  for (int g = 0; g < gpu_count; ++g) {
    if (numa[g] >= 0 && numa[g] < kMaxZones) {
      ++zone_gpus[numa[g]];
      zone_n = std::max(zone_n, numa[g] + 1);
    }
    refresh(g);
  }
}

GpuLedger::GpuFree GpuLedger::compute(int g) const {
  GpuFree f;
  if (monopoly[g] > 0) return f;
  int xpp = xcds_per_part(g);
  int64_t pm = part_mem(g);
  bool untouched = true;
  for (int s = offset[g]; s < offset[g + 1]; ++s) {
    const Slot& sl = slots[s];
    if (sl.exclusive > 0 || sl.used_mem > 0 || sl.mem_pods > 0) untouched = false;
    if (sl.exclusive == 0 && sl.used_mem == 0 && sl.mem_pods == 0) {
      ++f.free_slots;
      f.xcds += xpp;
    }
    if (sl.exclusive == 0) {
      f.mem += pm - sl.used_mem;
      f.max_slot_mem = std::max(f.max_slot_mem, pm - sl.used_mem);
    }
  }
  f.whole = parts[g] == 1 && untouched ? 1 : 0;
  return f;
}

void GpuLedger::refresh(int g) {
  GpuFree nf = compute(g);
  GpuFree& of = free[g];
  tot_whole += nf.whole - of.whole;
  tot_xcds += nf.xcds - of.xcds;
  tot_mem += nf.mem - of.mem;
  int z = numa[g];
  if (z >= 0 && z < kMaxZones) {
    zone_whole[z] += nf.whole - of.whole;
    zone_xcds[z] += nf.xcds - of.xcds;
    zone_mem[z] += nf.mem - of.mem;
  }
  of = nf;
}

void GpuLedger::apply(const GpuAssignment& a, int sign) {
  if (!a.valid() || gpu_count == 0) return;
  switch (a.kind) {
    case GpuAssignment::Kind::WholeGpu:
      for (int g : a.gpus)
        if (g >= 0 && g < gpu_count) {  // bounds-checked (Appendix C2)
          monopoly[g] += sign;
          refresh(g);
        }
      break;
    case GpuAssignment::Kind::Partition:
      for (auto [g, p] : a.partitions)
        if (g >= 0 && g < gpu_count && p >= 0 && p < parts[g]) {
          slots[offset[g] + p].exclusive += sign;
          refresh(g);
        }
      break;
    case GpuAssignment::Kind::Memory: {
      int g = a.gpus.empty() ? -1 : a.gpus[0];
      int p = a.partitions.empty() ? 0 : a.partitions[0].second;
      if (!a.partitions.empty()) g = a.partitions[0].first;
      if (g >= 0 && g < gpu_count && p >= 0 && p < parts[g]) {
        Slot& s = slots[offset[g] + p];
        s.used_mem += sign * a.memory;
        s.mem_pods += sign;
        refresh(g);
      }
      break;
    }
    default: break;
  }
}

bool GpuLedger::gpu_untouched(int g) const {
  if (monopoly[g] > 0) return false;
  for (int s = offset[g]; s < offset[g + 1]; ++s)
    if (slots[s].exclusive > 0 || slots[s].used_mem > 0 || slots[s].mem_pods > 0) return false;
  return true;
}

bool GpuLedger::slot_free(int g, int p) const {
  if (monopoly[g] > 0) return false;
  const Slot& s = slots[offset[g] + p];
  return s.exclusive == 0 && s.used_mem == 0 && s.mem_pods == 0;
}

// ------------------------------------------------------------- NodeInfo ----
namespace {
const std::string kEmpty;
bool has_affinity(const Pod& p) {
  return !p.pod_affinity_required.empty() || !p.pod_affinity_preferred.empty() ||
         !p.pod_anti_affinity_required.empty() || !p.pod_anti_affinity_preferred.empty();
}
}  // namespace

const std::string& NodeInfo::name() const { return node ? node->name() : kEmpty; }

void NodeInfo::set_node(const NodePtr& n) {
  node = n;
  allocatable = n->allocatable;
  gpu.init(*n);
  for (const auto& p : pods) gpu.apply(p->gpu, +1);
  ++generation;
}

void NodeInfo::add_pod(const PodPtr& p) {
  pods.push_back(p);
  pod_uid_hashes.push_back(std::hash<std::string>{}(p->uid()));
  if (has_affinity(*p)) pods_with_affinity.push_back(p);
  if (!p->pod_anti_affinity_required.empty()) pods_with_required_anti_affinity.push_back(p);
  requested += p->request();
  nonzero_requested += p->nonzero_request();
  for (const auto& port : p->host_ports) used_ports.emplace(port.host_ip, port.protocol, port.host_port);
  gpu.apply(p->gpu, +1);
  if (p->pg_key) {
    bool found = false;
    for (auto& [k, c] : pg_count)
      if (k == p->pg_key) {
        ++c;
        found = true;
        break;
      }
    if (!found) pg_count.emplace_back(p->pg_key, 1);
  }
  ++generation;
}

bool NodeInfo::remove_pod(const std::string& uid) {
  auto erase_from = [&](std::vector<PodPtr>& v) {
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i]->uid() == uid) {
        v[i] = v.back();
        v.pop_back();
        return true;
      }
    return false;
  };
  // One pass over the uid hashes finds the victim, which is swap-removed
  // (order is not semantic); the affinity lists are searched only when it
  // can be in them.
  PodPtr victim;
  const uint64_t h = std::hash<std::string>{}(uid);
  for (size_t i = 0; i < pods.size(); ++i)
    if (pod_uid_hashes[i] == h && pods[i]->uid() == uid) {
      victim = std::move(pods[i]);
      pods[i] = std::move(pods.back());
      pods.pop_back();
      pod_uid_hashes[i] = pod_uid_hashes.back();
      pod_uid_hashes.pop_back();
      break;
    }
  if (!victim) return false;
  if (has_affinity(*victim)) erase_from(pods_with_affinity);
  if (!victim->pod_anti_affinity_required.empty()) erase_from(pods_with_required_anti_affinity);
  requested -= victim->request();
  nonzero_requested -= victim->nonzero_request();
  for (const auto& port : victim->host_ports) used_ports.erase({port.host_ip, port.protocol, port.host_port});
  gpu.apply(victim->gpu, -1);
  if (victim->pg_key) {
    for (size_t i = 0; i < pg_count.size(); ++i)
      if (pg_count[i].first == victim->pg_key) {
        if (--pg_count[i].second <= 0) {
          pg_count[i] = pg_count.back();
          pg_count.pop_back();
        }
        break;
      }
  }
  ++generation;
  return true;
}

const PodPtr* NodeInfo::find_pod(const std::string& uid) const {
  const uint64_t h = std::hash<std::string>{}(uid);
  for (size_t i = 0; i < pods.size(); ++i)
    if (pod_uid_hashes[i] == h && pods[i]->uid() == uid) return &pods[i];
  return nullptr;
}

}  // namespace xsched

namespace xsched {

// ------------------------------------------------------- cache debugger ----
std::vector<std::string> GpuLedger::diff(const GpuLedger& o) const {
  std::vector<std::string> out;
  if (gpu_count != o.gpu_count || parts != o.parts) out.push_back("gpu.partitions");
  if (monopoly != o.monopoly) out.push_back("gpu.monopoly");
  if (slots.size() != o.slots.size()) {
    out.push_back("gpu.slots");
  } else {
    for (size_t i = 0; i < slots.size(); ++i)
      if (slots[i].exclusive != o.slots[i].exclusive || slots[i].used_mem != o.slots[i].used_mem ||
          slots[i].mem_pods != o.slots[i].mem_pods) {
        out.push_back("gpu.slots[" + std::to_string(i) + "]");
        break;
      }
  }
  if (tot_whole != o.tot_whole) out.push_back("gpu.free_whole");
  if (tot_xcds != o.tot_xcds) out.push_back("gpu.free_xcds");
  if (tot_mem != o.tot_mem) out.push_back("gpu.free_memory");
  for (int z = 0; z < kMaxZones; ++z)
    if (zone_gpus[z] != o.zone_gpus[z] || zone_whole[z] != o.zone_whole[z] || zone_xcds[z] != o.zone_xcds[z] ||
        zone_mem[z] != o.zone_mem[z]) {
      out.push_back("gpu.zone[" + std::to_string(z) + "]");
      break;
    }
  return out;
}

std::vector<std::string> NodeInfo::verify() const {
  std::vector<std::string> out;
  if (!node) return out;
  NodeInfo fresh;
  fresh.set_node(node);
  fresh.nrt = nrt;
  for (const auto& p : pods) fresh.add_pod(p);
  auto same_res = [](const Res& a, const Res& b) {
    for (int i = 0; i < kMaxRes; ++i)
      if (a.v[i] != b.v[i]) return false;
    return true;
  };
  if (!same_res(requested, fresh.requested)) out.push_back("requested");
  if (!same_res(nonzero_requested, fresh.nonzero_requested)) out.push_back("nonzero_requested");
  if (!same_res(allocatable, fresh.allocatable)) out.push_back("allocatable");
  if (used_ports != fresh.used_ports) out.push_back("used_ports");
  if (pods_with_affinity.size() != fresh.pods_with_affinity.size()) out.push_back("pods_with_affinity");
  if (pods_with_required_anti_affinity.size() != fresh.pods_with_required_anti_affinity.size())
    out.push_back("pods_with_required_anti_affinity");
  auto a = pg_count, b = fresh.pg_count;
  a.erase(std::remove_if(a.begin(), a.end(), [](const auto& kv) { return kv.second == 0; }), a.end());
  std::sort(a.begin(), a.end());
  std::sort(b.begin(), b.end());
  if (a != b) out.push_back("pg_count");
  for (auto& d : gpu.diff(fresh.gpu)) out.push_back(std::move(d));
  return out;
}

}  // namespace xsched
