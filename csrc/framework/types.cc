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

std::string Status::message() const {
  std::string s;
  for (size_t i = 0; i < reasons_.size(); ++i) {
    if (i) s += ", ";
    s += reasons_[i];
  }
  return s;
}

// ----------------------------------------------------------- CycleState ----
std::shared_ptr<StateData> CycleState::read(const std::string& key) const {
  std::lock_guard<std::mutex> g(mu_);
  for (const auto& kv : kv_)
    if (kv.first == key) return kv.second;
  return nullptr;
}

void CycleState::write(const std::string& key, std::shared_ptr<StateData> v) {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& kv : kv_)
    if (kv.first == key) {
      kv.second = std::move(v);
      return;
    }
  kv_.emplace_back(key, std::move(v));
}

void CycleState::erase(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  kv_.erase(std::remove_if(kv_.begin(), kv_.end(), [&](const auto& kv) { return kv.first == key; }), kv_.end());
}

std::shared_ptr<CycleState> CycleState::clone() const {
  auto c = std::make_shared<CycleState>();
  std::lock_guard<std::mutex> g(mu_);
  for (const auto& kv : kv_) {
    if (!kv.second) continue;
    auto cl = kv.second->clone();
    c->kv_.emplace_back(kv.first, cl ? cl : kv.second);
  }
  c->record_metrics = record_metrics;
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
}

void GpuLedger::apply(const GpuAssignment& a, int sign) {
  if (!a.valid() || gpu_count == 0) return;
  switch (a.kind) {
    case GpuAssignment::Kind::WholeGpu:
      for (int g : a.gpus)
        if (g >= 0 && g < gpu_count) monopoly[g] += sign;  // bounds-checked (Appendix C2)
      break;
    case GpuAssignment::Kind::Partition:
      for (auto [g, p] : a.partitions)
        if (g >= 0 && g < gpu_count && p >= 0 && p < parts[g]) slots[offset[g] + p].exclusive += sign;
      break;
    case GpuAssignment::Kind::Memory: {
      int g = a.gpus.empty() ? -1 : a.gpus[0];
      int p = a.partitions.empty() ? 0 : a.partitions[0].second;
      if (!a.partitions.empty()) g = a.partitions[0].first;
      if (g >= 0 && g < gpu_count && p >= 0 && p < parts[g]) {
        Slot& s = slots[offset[g] + p];
        s.used_mem += sign * a.memory;
        s.mem_pods += sign;
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

int GpuLedger::free_gpus() const {
  int n = 0;
  for (int g = 0; g < gpu_count; ++g) n += whole_gpu_free(g) ? 1 : 0;
  return n;
}

int64_t GpuLedger::free_memory() const {
  int64_t free = 0;
  for (int g = 0; g < gpu_count; ++g) {
    if (monopoly[g] > 0) continue;
    int64_t pm = part_mem(g);
    for (int s = offset[g]; s < offset[g + 1]; ++s)
      if (slots[s].exclusive == 0) free += pm - slots[s].used_mem;
  }
  return free;
}

int GpuLedger::free_xcds() const {
  int n = 0;
  for (int g = 0; g < gpu_count; ++g) {
    if (monopoly[g] > 0) continue;
    for (int p = 0; p < parts[g]; ++p)
      if (slot_free(g, p)) n += xcds_per_part(g);
  }
  return n;
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
  if (has_affinity(*p)) pods_with_affinity.push_back(p);
  if (!p->pod_anti_affinity_required.empty()) pods_with_required_anti_affinity.push_back(p);
  requested += p->request;
  nonzero_requested += p->nonzero_request;
  for (const auto& port : p->host_ports) used_ports.emplace(port.host_ip, port.protocol, port.host_port);
  gpu.apply(p->gpu, +1);
  if (!p->pod_group.empty()) ++pg_count[p->pg_full_name()];
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
  PodPtr victim;
  for (const auto& p : pods)
    if (p->uid() == uid) {
      victim = p;
      break;
    }
  if (!victim) return false;
  // Keep `pods` order stable-ish: swap-remove is fine (order is not semantic).
  erase_from(pods);
  erase_from(pods_with_affinity);
  erase_from(pods_with_required_anti_affinity);
  requested -= victim->request;
  nonzero_requested -= victim->nonzero_request;
  for (const auto& port : victim->host_ports) used_ports.erase({port.host_ip, port.protocol, port.host_port});
  gpu.apply(victim->gpu, -1);
  if (!victim->pod_group.empty()) {
    auto it = pg_count.find(victim->pg_full_name());
    if (it != pg_count.end() && --it->second <= 0) pg_count.erase(it);
  }
  ++generation;
  return true;
}

const PodPtr* NodeInfo::find_pod(const std::string& uid) const {
  for (const auto& p : pods)
    if (p->uid() == uid) return &p;
  return nullptr;
}

}  // namespace xsched
