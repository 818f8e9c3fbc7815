// Dense resource vectors (the scheduler's framework.Resource equivalent).
//
// The reference's framework.Resource (vendor/k8s.io/kubernetes/pkg/scheduler/
// framework/types.go: MilliCPU, Memory, EphemeralStorage, AllowedPodNumber,
// ScalarResources map) is a struct-plus-map. Here every resource name is
// interned to a small id and a resource vector is a fixed array + a presence
// mask, so Fit checks and NodeInfo accounting are branch-light loops over set
// bits instead of map walks. The presence mask preserves Go's "key absent vs
// zero" distinction that ElasticQuota's cmp2 relies on
// (pkg/capacityscheduling/elasticquota.go:165-181).
#pragma once

#include <array>
#include <cstdint>
#include <mutex>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "common/json.h"
#include "common/quantity.h"

namespace xsched {

constexpr int kMaxRes = 48;
enum ResId : int { kCPU = 0, kMemory = 1, kEphemeral = 2, kPods = 3 };

class ResourceRegistry {
 public:
  static ResourceRegistry& get();
  int id(std::string_view name);          // interns (throws when full)
  int find(std::string_view name) const;  // -1 when unknown
  std::string name(int id) const;
  int size() const;
  // Native resources per k8s (cpu, memory, ephemeral-storage, pods, hugepages-*).
  // Flags are fixed at interning time, so these are lock-free.
  bool is_native(int id) const { return id >= 0 && id < kMaxRes && (flags_[id] & kNative); }
  bool is_hugepages(int id) const { return id >= 0 && id < kMaxRes && (flags_[id] & kHuge); }

 private:
  int id_locked(std::string_view name);
  enum : uint8_t { kNative = 1, kHuge = 2 };
  static uint8_t flags_for(std::string_view name);
  ResourceRegistry();
  std::array<uint8_t, kMaxRes> flags_{};
  mutable std::mutex mu_;
  std::vector<std::string> names_;
  std::unordered_map<std::string, int> ids_;
};

inline int res_id(std::string_view name) { return ResourceRegistry::get().id(name); }

struct Res {
  uint64_t mask = 0;
  std::array<int64_t, kMaxRes> v{};

  bool has(int id) const { return (mask >> id) & 1u; }
  int64_t get(int id) const { return v[id]; }
  void set(int id, int64_t x) { v[id] = x; mask |= (uint64_t{1} << id); }
  void add_to(int id, int64_t x) { v[id] += x; mask |= (uint64_t{1} << id); }
  void clear() { mask = 0; v.fill(0); }
  bool empty() const { return mask == 0; }

  Res& operator+=(const Res& o) {
    for (uint64_t m = o.mask; m; m &= m - 1) {
      int i = __builtin_ctzll(m);
      v[i] += o.v[i];
    }
    mask |= o.mask;
    return *this;
  }
  Res& operator-=(const Res& o) {
    for (uint64_t m = o.mask; m; m &= m - 1) {
      int i = __builtin_ctzll(m);
      v[i] -= o.v[i];
    }
    mask |= o.mask;
    return *this;
  }
  // Elementwise max (init-container semantics of computePodResourceRequest).
  void set_max(const Res& o) {
    for (uint64_t m = o.mask; m; m &= m - 1) {
      int i = __builtin_ctzll(m);
      if (!has(i) || o.v[i] > v[i]) v[i] = o.v[i];
    }
    mask |= o.mask;
  }
  bool operator==(const Res& o) const {
    uint64_t m = mask | o.mask;
    for (; m; m &= m - 1) {
      int i = __builtin_ctzll(m);
      if (v[i] != o.v[i]) return false;
    }
    return true;
  }

  // ResourceList JSON ({"cpu":"500m","memory":"1Gi",...}) <-> Res.
  static Res from_json(const Json& rl);
  Json to_json() const;
  std::string debug() const;
};

// Parse one quantity into the integer unit the scheduler uses for resource
// `id`: milli-CPU for cpu, Value() (rounded up) for everything else.
int64_t quantity_to_res_units(int id, const Quantity& q);
Quantity res_units_to_quantity(int id, int64_t v);

}  // namespace xsched
