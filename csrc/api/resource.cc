#include "api/resource.h"

#include <stdexcept>

namespace xsched {

ResourceRegistry& ResourceRegistry::get() {
  static ResourceRegistry* r = new ResourceRegistry();
  return *r;
}

uint8_t ResourceRegistry::flags_for(std::string_view n) {
  uint8_t f = 0;
  // v1helper.IsNativeResource: no domain prefix or the kubernetes.io/ domain.
  if (n.find('/') == std::string_view::npos || n.rfind("kubernetes.io/", 0) == 0) f |= kNative;
  if (n.rfind("hugepages-", 0) == 0) f |= kHuge;
  return f;
}

ResourceRegistry::ResourceRegistry() {
  for (const char* n : {"cpu", "memory", "ephemeral-storage", "pods"}) {
    flags_[names_.size()] = flags_for(n);
    ids_.emplace(n, static_cast<int>(names_.size()));
    names_.emplace_back(n);
  }
}

int ResourceRegistry::id(std::string_view name) {
  // Ids never change once assigned: a per-thread cache of the names a thread
  // saw skips the lock and the key allocation (pod parses run on several
  // threads and ask for the same handful of names).
  struct Seen {
    const ResourceRegistry* reg;
    std::string name;
    int id;
  };
  thread_local std::vector<Seen> seen;
  for (const auto& e : seen)
    if (e.reg == this && e.name == name) return e.id;
  const int id = id_locked(name);
  if (seen.size() < 32) seen.push_back(Seen{this, std::string(name), id});
  return id;
}

int ResourceRegistry::id_locked(std::string_view name) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = ids_.find(std::string(name));
  if (it != ids_.end()) return it->second;
  if (static_cast<int>(names_.size()) >= kMaxRes)
    throw std::runtime_error("too many distinct resource names (max " + std::to_string(kMaxRes) + ")");
  int id = static_cast<int>(names_.size());
  flags_[id] = flags_for(name);
  names_.emplace_back(name);
  ids_.emplace(std::string(name), id);
  return id;
}

int ResourceRegistry::find(std::string_view name) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = ids_.find(std::string(name));
  return it == ids_.end() ? -1 : it->second;
}

std::string ResourceRegistry::name(int id) const {
  std::lock_guard<std::mutex> g(mu_);
  return id >= 0 && id < static_cast<int>(names_.size()) ? names_[id] : std::string();
}

int ResourceRegistry::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return static_cast<int>(names_.size());
}

int64_t quantity_to_res_units(int id, const Quantity& q) {
  return id == kCPU ? q.milli_value() : q.value();
}

Quantity res_units_to_quantity(int id, int64_t v) {
  if (id == kCPU) return Quantity::from_milli(v);
  if (id == kMemory || id == kEphemeral || ResourceRegistry::get().is_hugepages(id))
    return Quantity::from_int(v, Quantity::Format::BinarySI);
  return Quantity::from_int(v);
}

Res Res::from_json(const Json& rl) {
  Res r;
  for (const auto& kv : rl.members()) {
    int id = res_id(kv.first);
    Quantity q;
    if (kv.second.is_string()) {
      q = Quantity::parse(kv.second.as_string());
    } else if (kv.second.is_int()) {
      q = Quantity::from_int(kv.second.as_int());
    } else if (kv.second.is_number()) {
      q = Quantity::parse(std::to_string(kv.second.as_double()));
    } else {
      continue;
    }
    r.set(id, quantity_to_res_units(id, q));
  }
  return r;
}

Json Res::to_json() const {
  Json o = Json::object();
  auto& reg = ResourceRegistry::get();
  for (uint64_t m = mask; m; m &= m - 1) {
    int i = __builtin_ctzll(m);
    o.set(reg.name(i), Json(res_units_to_quantity(i, v[i]).str()));
  }
  return o;
}

std::string Res::debug() const {
  std::string s = "{";
  auto& reg = ResourceRegistry::get();
  bool first = true;
  for (uint64_t m = mask; m; m &= m - 1) {
    int i = __builtin_ctzll(m);
    if (!first) s += ", ";
    first = false;
    s += reg.name(i) + ":" + std::to_string(v[i]);
  }
  return s + "}";
}

}  // namespace xsched
