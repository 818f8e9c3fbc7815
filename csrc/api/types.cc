#include "api/types.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <unordered_set>

#include "api/storage.h"

namespace xsched {

// ---------------------------------------------------------------- time ----
namespace {
int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = static_cast<unsigned>(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + static_cast<int64_t>(doe) - 719468;
}
void civil_from_days(int64_t z, int64_t* y, unsigned* m, unsigned* d) {
  z += 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const unsigned doe = static_cast<unsigned>(z - era * 146097);
  const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const unsigned mp = (5 * doy + 2) / 153;
  *d = doy - (153 * mp + 2) / 5 + 1;
  *m = mp < 10 ? mp + 3 : mp - 9;
  *y = static_cast<int64_t>(yoe) + era * 400 + (*m <= 2);
}
}  // namespace

MicroTime parse_rfc3339(const std::string& s) {
  if (s.size() < 19) return 0;
  // Fixed-width "YYYY-MM-DDTHH:MM:SS" read digit by digit (every watched Pod
  // carries a creationTimestamp; sscanf was a visible share of parsing).
  auto num = [&](size_t at, size_t width, int* out) {
    int v = 0;
    for (size_t k = at; k < at + width; ++k) {
      if (s[k] < '0' || s[k] > '9') return false;
      v = v * 10 + (s[k] - '0');
    }
    *out = v;
    return true;
  };
  int Y, M, D, h, mi, sec;
  if (!num(0, 4, &Y) || s[4] != '-' || !num(5, 2, &M) || s[7] != '-' || !num(8, 2, &D) ||
      (s[10] != 'T' && s[10] != 't' && s[10] != ' ') || !num(11, 2, &h) || s[13] != ':' || !num(14, 2, &mi) ||
      s[16] != ':' || !num(17, 2, &sec))
    return 0;
  size_t i = 19;
  int64_t frac_us = 0;
  if (i < s.size() && s[i] == '.') {
    ++i;
    int digits = 0;
    while (i < s.size() && s[i] >= '0' && s[i] <= '9') {
      if (digits < 6) {
        frac_us = frac_us * 10 + (s[i] - '0');
        ++digits;
      }
      ++i;
    }
    while (digits < 6) { frac_us *= 10; ++digits; }
  }
  int64_t offset_s = 0;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) {
    int oh = 0, om = 0;
    std::sscanf(s.c_str() + i + 1, "%2d:%2d", &oh, &om);
    offset_s = (oh * 3600 + om * 60) * (s[i] == '-' ? -1 : 1);
  }
  int64_t days = days_from_civil(Y, static_cast<unsigned>(M), static_cast<unsigned>(D));
  int64_t secs = days * 86400 + h * 3600 + mi * 60 + sec - offset_s;
  return secs * 1000000 + frac_us;
}

std::string format_rfc3339(MicroTime t) {
  int64_t secs = t >= 0 ? t / 1000000 : (t - 999999) / 1000000;
  int64_t us = t - secs * 1000000;
  int64_t days = secs >= 0 ? secs / 86400 : (secs - 86399) / 86400;
  int64_t rem = secs - days * 86400;
  int64_t y;
  unsigned m, d;
  civil_from_days(days, &y, &m, &d);
  char buf[64];
  if (us == 0)
    std::snprintf(buf, sizeof buf, "%04lld-%02u-%02uT%02lld:%02lld:%02lldZ", static_cast<long long>(y), m, d,
                  static_cast<long long>(rem / 3600), static_cast<long long>((rem / 60) % 60),
                  static_cast<long long>(rem % 60));
  else
    std::snprintf(buf, sizeof buf, "%04lld-%02u-%02uT%02lld:%02lld:%02lld.%06lldZ", static_cast<long long>(y), m, d,
                  static_cast<long long>(rem / 3600), static_cast<long long>((rem / 60) % 60),
                  static_cast<long long>(rem % 60), static_cast<long long>(us));
  return buf;
}

MicroTime wall_now_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

// ---------------------------------------------------------------- maps ----
const std::string* strmap_get(const StrMap& m, std::string_view k) {
  for (const auto& kv : m)
    if (kv.first == k) return &kv.second;
  return nullptr;
}

StrMap strmap_from_json(const Json& j) {
  StrMap m;
  m.reserve(j.size());
  for (const auto& kv : j.members()) m.emplace_back(kv.first, kv.second.as_string());
  return m;
}

ObjectMeta ObjectMeta::from_json(const Json& obj) {
  ObjectMeta m;
  const Json& md = obj["metadata"];
  m.ns = md["namespace"].as_string();
  m.name = md["name"].as_string();
  m.uid = md["uid"].as_string();
  const Json& rv = md["resourceVersion"];
  m.resource_version = rv.is_string() ? std::atoll(rv.as_string().c_str()) : rv.as_int();
  m.labels = strmap_from_json(md["labels"]);
  m.annotations = strmap_from_json(md["annotations"]);
  if (md["creationTimestamp"].is_string()) m.creation = parse_rfc3339(md["creationTimestamp"].as_string());
  if (md["deletionTimestamp"].is_string()) m.deletion = parse_rfc3339(md["deletionTimestamp"].as_string());
  return m;
}

// ----------------------------------------------------------- selectors ----
namespace {
SelOp parse_op(const std::string& s) {
  if (s == "NotIn") return SelOp::NotIn;
  if (s == "Exists") return SelOp::Exists;
  if (s == "DoesNotExist") return SelOp::DoesNotExist;
  if (s == "Gt") return SelOp::Gt;
  if (s == "Lt") return SelOp::Lt;
  return SelOp::In;
}
std::vector<SelectorRequirement> parse_reqs(const Json& arr) {
  std::vector<SelectorRequirement> out;
  for (const auto& e : arr.items()) {
    SelectorRequirement r;
    r.key = e["key"].as_string();
    r.op = parse_op(e["operator"].as_string());
    for (const auto& v : e["values"].items()) r.values.push_back(v.as_string());
    out.push_back(std::move(r));
  }
  return out;
}
}  // namespace

bool match_requirement(const SelectorRequirement& r, const StrMap& labels) {
  const std::string* v = strmap_get(labels, r.key);
  switch (r.op) {
    case SelOp::In:
      return v && std::find(r.values.begin(), r.values.end(), *v) != r.values.end();
    case SelOp::NotIn:
      return !v || std::find(r.values.begin(), r.values.end(), *v) == r.values.end();
    case SelOp::Exists:
      return v != nullptr;
    case SelOp::DoesNotExist:
      return v == nullptr;
    case SelOp::Gt:
    case SelOp::Lt: {
      if (!v || r.values.size() != 1) return false;
      char* e1 = nullptr;
      char* e2 = nullptr;
      long long a = std::strtoll(v->c_str(), &e1, 10);
      long long b = std::strtoll(r.values[0].c_str(), &e2, 10);
      if (*e1 || *e2) return false;
      return r.op == SelOp::Gt ? a > b : a < b;
    }
  }
  return false;
}

bool LabelSelector::matches(const StrMap& labels) const {
  if (!present) return false;
  for (const auto& kv : match_labels) {
    const std::string* v = strmap_get(labels, kv.first);
    if (!v || *v != kv.second) return false;
  }
  for (const auto& r : exprs)
    if (!match_requirement(r, labels)) return false;
  return true;
}

LabelSelector LabelSelector::from_json(const Json* j) {
  LabelSelector s;
  if (!j || j->is_null()) return s;
  s.present = true;
  s.match_labels = strmap_from_json((*j)["matchLabels"]);
  s.exprs = parse_reqs((*j)["matchExpressions"]);
  return s;
}

bool Toleration::tolerates(const Taint& t) const {
  // v1helper ToleratesTaint semantics.
  if (!effect.empty() && effect != t.effect) return false;
  if (!key.empty() && key != t.key) return false;
  if (op == "Exists") return true;
  if (op == "Equal" || op.empty()) return value == t.value;
  return false;
}

// ----------------------------------------------------------------- Pod ----
namespace {
Container parse_container(const Json& c) {
  Container out;
  out.name = c["name"].as_string();
  out.image = c["image"].as_string();
  const Json& res = c["resources"];
  out.limits = Res::from_json(res["limits"]);
  out.requests = Res::from_json(res["requests"]);
  // apiserver defaulting: a limit without a request defaults the request.
  for (uint64_t m = out.limits.mask & ~out.requests.mask; m; m &= m - 1) {
    int i = __builtin_ctzll(m);
    out.requests.set(i, out.limits.v[i]);
  }
  for (const auto& p : c["ports"].items()) {
    ContainerPort cp;
    cp.host_port = static_cast<int32_t>(p["hostPort"].as_int(0));
    cp.protocol = p["protocol"].str_or("TCP");
    cp.host_ip = p["hostIP"].str_or("0.0.0.0");
    out.ports.push_back(cp);
  }
  return out;
}

NodeSelectorTerm parse_term(const Json& t) {
  NodeSelectorTerm term;
  term.match_expressions = parse_reqs(t["matchExpressions"]);
  term.match_fields = parse_reqs(t["matchFields"]);
  return term;
}

PodAffinityTerm parse_pod_affinity_term(const Json& t) {
  PodAffinityTerm out;
  out.selector = LabelSelector::from_json(t.get("labelSelector"));
  for (const auto& n : t["namespaces"].items()) out.namespaces.push_back(n.as_string());
  out.namespace_selector = LabelSelector::from_json(t.get("namespaceSelector"));
  out.topology_key = t["topologyKey"].as_string();
  return out;
}

void parse_pod_affinity(const Json& a, std::vector<PodAffinityTerm>* req, std::vector<WeightedPodAffinityTerm>* pref) {
  for (const auto& t : a["requiredDuringSchedulingIgnoredDuringExecution"].items())
    req->push_back(parse_pod_affinity_term(t));
  for (const auto& t : a["preferredDuringSchedulingIgnoredDuringExecution"].items()) {
    WeightedPodAffinityTerm w;
    w.weight = static_cast<int32_t>(t["weight"].as_int());
    w.term = parse_pod_affinity_term(t["podAffinityTerm"]);
    pref->push_back(std::move(w));
  }
}

// Defaults from pkg/scheduler/util/non_zero.go (DefaultMilliCPURequest=100m,
// DefaultMemoryRequest=200MB).
constexpr int64_t kDefaultMilliCPU = 100;
constexpr int64_t kDefaultMemory = 200 * 1024 * 1024;

QoS compute_qos(const Pod& p) {
  // v1qos.GetPodQOS over cpu/memory.
  bool any = false;
  bool guaranteed = true;
  auto visit = [&](const Container& c) {
    for (int id : {static_cast<int>(kCPU), static_cast<int>(kMemory)}) {
      bool has_req = c.requests.has(id) && c.requests.get(id) != 0;
      bool has_lim = c.limits.has(id) && c.limits.get(id) != 0;
      if (has_req || has_lim) any = true;
      if (!has_lim) guaranteed = false;
      else if (has_req && c.requests.get(id) != c.limits.get(id)) guaranteed = false;
    }
  };
  for (const auto& c : p.containers) visit(c);
  for (const auto& c : p.init_containers) visit(c);
  if (!any) return QoS::BestEffort;
  return guaranteed ? QoS::Guaranteed : QoS::Burstable;
}

std::vector<int> parse_int_list(const std::string& s) {
  std::vector<int> out;
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    std::string tok = s.substr(i, j - i);
    char* e = nullptr;
    long v = std::strtol(tok.c_str(), &e, 10);
    if (!tok.empty() && e && *e == '\0' && v >= 0) out.push_back(static_cast<int>(v));
    else return {};
    i = j + 1;
  }
  return out;
}
}  // namespace

void Pod::recompute_gpu_assignment(const GpuNames& gn) {
  gpu = GpuAssignment{};
  const std::string* idx = meta.annotation(gn.index_annotation);
  if (!idx) return;
  std::vector<int> gpus = parse_int_list(*idx);
  if (gpus.empty()) return;  // unparsable annotation: skipped (gpu_node.go:91-96)
  std::vector<std::pair<int, int>> parts;
  if (const std::string* ps = meta.annotation(gn.partition_annotation)) {
    size_t i = 0;
    const std::string& s = *ps;
    while (i < s.size()) {
      size_t j = s.find(',', i);
      if (j == std::string::npos) j = s.size();
      std::string tok = s.substr(i, j - i);
      size_t c = tok.find(':');
      if (c != std::string::npos) {
        parts.emplace_back(std::atoi(tok.substr(0, c).c_str()), std::atoi(tok.substr(c + 1).c_str()));
      }
      i = j + 1;
    }
  }
  set_gpu_assignment(std::move(gpus), std::move(parts), gn);
}

void Pod::set_gpu_assignment(std::vector<int> gpus, std::vector<std::pair<int, int>> parts, const GpuNames& gn) {
  gpu = GpuAssignment{};
  if (gpus.empty()) return;
  int gid = gn.gpu_id(), mid = gn.memory_id(), xid = gn.xcd_id();
  const Res& limits = limit_sum();
  if (limits.has(gid) && limits.get(gid) > 0) {
    gpu.kind = GpuAssignment::Kind::WholeGpu;
  } else if (limits.has(xid) && limits.get(xid) > 0) {
    gpu.kind = GpuAssignment::Kind::Partition;
  } else if (limits.has(mid)) {
    gpu.kind = GpuAssignment::Kind::Memory;
    gpu.memory = limits.get(mid);
  } else {
    return;
  }
  gpu.gpus = std::move(gpus);
  gpu.partitions = std::move(parts);
}

const std::string& IStr::intern(std::string_view v) {
  // The values almost every pod carries skip the table lock.
  static const std::string* kCommon[] = {new std::string(kDefaultSchedulerName), new std::string("PreemptLowerPriority"),
                                         new std::string("")};
  for (const std::string* c : kCommon)
    if (*c == v) return *c;
  static std::mutex mu;
  static auto* table = new std::unordered_set<std::string>();  // never freed: IStr pointers outlive statics
  std::lock_guard<std::mutex> g(mu);
  return *table->emplace(v).first;
}

uint64_t pg_key_of(std::string_view full) {
  uint64_t h = 1469598103934665603ULL;
  for (unsigned char c : full) {
    h ^= c;
    h *= 1099511628211ULL;
  }
  return h ? h : 1;
}

std::shared_ptr<Pod> Pod::from_json(const Json& obj, const GpuNames& gn) {
  auto p = std::make_shared<Pod>();
  p->meta = ObjectMeta::from_json(obj);
  const Json& spec = obj["spec"];
  const Json& status = obj["status"];
  p->spec_hash = json_hash(spec, 1469598103934665603ULL, "nodeName");
  if (spec["nodeName"].as_string().empty()) {  // only pending pods are ever scheduled
    const Json& md = obj["metadata"];
    uint64_t h = json_hash(md["namespace"], p->spec_hash);
    p->template_hash = json_hash(md["annotations"], h);
  }
  if (spec["schedulerName"].is_string()) p->scheduler_name = spec["schedulerName"].as_string();
  p->node_name = spec["nodeName"].as_string();
  p->priority_class_name = spec["priorityClassName"].as_string();
  p->priority = static_cast<int32_t>(spec["priority"].as_int(0));
  if (spec["preemptionPolicy"].is_string()) p->preemption_policy = spec["preemptionPolicy"].as_string();
  {
    std::vector<Container> cs, ics;
    for (const auto& c : spec["containers"].items()) cs.push_back(parse_container(c));
    for (const auto& c : spec["initContainers"].items()) ics.push_back(parse_container(c));
    p->containers = std::move(cs);
    p->init_containers = std::move(ics);
  }
  p->volumes = parse_pod_volumes(spec, p->meta.name);
  auto res = std::make_shared<PodRes>();
  res->overhead = Res::from_json(spec["overhead"]);
  p->node_selector = strmap_from_json(spec["nodeSelector"]);
  if (const Json* na = spec.path({"affinity", "nodeAffinity"})) {
    if (const Json* req = na->get("requiredDuringSchedulingIgnoredDuringExecution")) {
      p->has_required_node_affinity = true;
      for (const auto& t : (*req)["nodeSelectorTerms"].items()) p->required_node_terms.push_back(parse_term(t));
    }
    for (const auto& t : (*na)["preferredDuringSchedulingIgnoredDuringExecution"].items()) {
      PreferredSchedulingTerm pt;
      pt.weight = static_cast<int32_t>(t["weight"].as_int());
      pt.pref = parse_term(t["preference"]);
      p->preferred_node_terms.push_back(std::move(pt));
    }
  }
  if (const Json* pa = spec.path({"affinity", "podAffinity"}))
    parse_pod_affinity(*pa, &p->pod_affinity_required, &p->pod_affinity_preferred);
  if (const Json* paa = spec.path({"affinity", "podAntiAffinity"}))
    parse_pod_affinity(*paa, &p->pod_anti_affinity_required, &p->pod_anti_affinity_preferred);
  for (const auto& c : spec["topologySpreadConstraints"].items()) {
    TopologySpreadConstraint tc;
    tc.max_skew = static_cast<int32_t>(c["maxSkew"].as_int(1));
    tc.topology_key = c["topologyKey"].as_string();
    tc.hard = c["whenUnsatisfiable"].str_or("DoNotSchedule") != "ScheduleAnyway";
    tc.selector = LabelSelector::from_json(c.get("labelSelector"));
    p->spread_constraints.push_back(std::move(tc));
  }
  for (const auto& t : spec["tolerations"].items()) {
    Toleration tol;
    tol.key = t["key"].as_string();
    tol.op = t["operator"].str_or("Equal");
    tol.value = t["value"].as_string();
    tol.effect = t["effect"].as_string();
    if (t["tolerationSeconds"].is_number()) tol.toleration_seconds = t["tolerationSeconds"].as_int();
    p->tolerations.push_back(std::move(tol));
  }
  if (status["phase"].is_string()) p->phase = status["phase"].as_string();
  p->nominated_node_name = status["nominatedNodeName"].as_string();
  if (status["startTime"].is_string()) p->start_time = parse_rfc3339(status["startTime"].as_string());
  for (const auto& c : status["conditions"].items())
    if (c["type"].as_string() == "PodScheduled" && c["status"].as_string() == "True")
      p->scheduled_at = parse_rfc3339(c["lastTransitionTime"].as_string());

  // Derived request/limit vectors.
  Res sum;
  for (const auto& c : p->containers) {
    sum += c.requests;
    res->limit_sum += c.limits;
    Res nz;
    nz.set(kCPU, c.requests.has(kCPU) && c.requests.get(kCPU) != 0 ? c.requests.get(kCPU) : kDefaultMilliCPU);
    nz.set(kMemory, c.requests.has(kMemory) && c.requests.get(kMemory) != 0 ? c.requests.get(kMemory) : kDefaultMemory);
    res->nonzero_request += nz;
    for (const auto& port : c.ports)
      if (port.host_port > 0) p->host_ports.push_back(port);
  }
  if (p->containers.empty()) {
    res->nonzero_request.set(kCPU, 0);
    res->nonzero_request.set(kMemory, 0);
  }
  for (const auto& c : p->init_containers) {
    sum.set_max(c.requests);
    Res nz;
    nz.set(kCPU, c.requests.has(kCPU) && c.requests.get(kCPU) != 0 ? c.requests.get(kCPU) : kDefaultMilliCPU);
    nz.set(kMemory, c.requests.has(kMemory) && c.requests.get(kMemory) != 0 ? c.requests.get(kMemory) : kDefaultMemory);
    res->nonzero_request.set_max(nz);
  }
  sum += res->overhead;
  res->nonzero_request += res->overhead;
  res->request = sum;
  p->res = std::move(res);
  p->qos = compute_qos(*p);
  if (const std::string* pg = p->meta.label(kPodGroupLabel)) {
    p->pod_group = *pg;
    p->pg_key = pg_key_of(p->pg_full_name());
  }
  p->gpu_demand = compute_gpu_demand(*p, gn);
  p->recompute_gpu_assignment(gn);
  return p;
}

// ---------------------------------------------------------------- Node ----
int partitions_for_mode(const std::string& mode) {
  std::string m;
  for (char c : mode) m.push_back(static_cast<char>(std::tolower(static_cast<unsigned char>(c))));
  if (m == "spx") return 1;
  if (m == "dpx") return 2;
  if (m == "qpx") return 4;
  if (m == "cpx") return 8;
  return 0;
}

bool node_selector_term_matches(const NodeSelectorTerm& t, const Node& n) {
  if (t.match_expressions.empty() && t.match_fields.empty()) return false;
  for (const auto& r : t.match_expressions)
    if (!match_requirement(r, n.meta.labels)) return false;
  for (const auto& r : t.match_fields) {
    if (r.key != "metadata.name") return false;
    StrMap f{{"metadata.name", n.name()}};
    if (!match_requirement(r, f)) return false;
  }
  return true;
}

bool pod_matches_node_selector_and_affinity(const Pod& p, const Node& n) {
  for (const auto& kv : p.node_selector) {
    const std::string* v = n.meta.label(kv.first);
    if (!v || *v != kv.second) return false;
  }
  if (!p.has_required_node_affinity) return true;
  for (const auto& t : p.required_node_terms)
    if (node_selector_term_matches(t, n)) return true;
  return false;
}

std::shared_ptr<Node> Node::from_json(const Json& obj, const GpuNames& gn) {
  auto n = std::make_shared<Node>();
  n->meta = ObjectMeta::from_json(obj);
  const Json& spec = obj["spec"];
  const Json& status = obj["status"];
  n->allocatable = Res::from_json(status["allocatable"]);
  n->capacity = Res::from_json(status["capacity"]);
  if (n->allocatable.empty()) n->allocatable = n->capacity;
  n->unschedulable = spec["unschedulable"].as_bool(false);
  for (const auto& t : spec["taints"].items()) {
    n->taints.push_back(Taint{t["key"].as_string(), t["value"].as_string(), t["effect"].as_string()});
    if (n->taints.back().effect == "PreferNoSchedule") n->has_prefer_no_schedule = true;
  }
  if (const std::string* h = n->meta.label(kHostnameLabel)) n->foreign_hostname = *h != n->meta.name;
  for (const auto& im : status["images"].items()) {
    ContainerImage ci;
    for (const auto& nm : im["names"].items()) ci.names.push_back(nm.as_string());
    ci.size_bytes = im["sizeBytes"].as_int(0);
    for (const auto& nm : ci.names) n->image_sizes.emplace(nm, ci.size_bytes);
    n->images.push_back(std::move(ci));
  }
  int gid = gn.gpu_id();
  n->gpu_count = n->allocatable.has(gid) ? static_cast<int>(n->allocatable.get(gid)) : 0;
  int parts = 1;
  if (const std::string* mode = n->meta.label(gn.partition_label)) {
    int p = partitions_for_mode(*mode);
    if (p > 0) parts = p;
  }
  n->gpu_partitions.assign(n->gpu_count, parts);
  n->gpu_numa.assign(n->gpu_count, -1);
  int mid = gn.memory_id();
  if (n->gpu_count > 0 && n->allocatable.has(mid))  // homogeneous split (gpu_node.go:51-55)
    n->gpu_memory_per_gpu = n->allocatable.get(mid) / n->gpu_count;
  if (const std::string* topo = n->meta.annotation(gn.topology_annotation)) {
    try {
      Json t = Json::parse(*topo);
      for (const auto& g : t["gpus"].items()) {
        int idx = static_cast<int>(g["index"].as_int(-1));
        if (idx < 0 || idx >= n->gpu_count) continue;
        if (g["partitions"].is_number()) {
          int p = static_cast<int>(g["partitions"].as_int());
          if (p == 1 || p == 2 || p == 4 || p == 8) n->gpu_partitions[idx] = p;
        } else if (g["partitionMode"].is_string()) {
          int p = partitions_for_mode(g["partitionMode"].as_string());
          if (p > 0) n->gpu_partitions[idx] = p;
        }
        if (g["numa"].is_number()) n->gpu_numa[idx] = static_cast<int>(g["numa"].as_int());
      }
    } catch (const JsonError&) {
      // malformed topology annotation: keep label/allocatable-derived model
    }
  }
  return n;
}

// ------------------------------------------------------------ CRD types ----
std::shared_ptr<PodGroup> PodGroup::from_json(const Json& obj) {
  auto pg = std::make_shared<PodGroup>();
  pg->meta = ObjectMeta::from_json(obj);
  const Json& spec = obj["spec"];
  const Json& st = obj["status"];
  pg->min_member = static_cast<int32_t>(spec["minMember"].as_int(0));
  if (const Json* mr = spec.get("minResources"); mr && mr->is_object()) {
    pg->has_min_resources = true;
    pg->min_resources = Res::from_json(*mr);
  }
  if (spec["scheduleTimeoutSeconds"].is_number())
    pg->schedule_timeout_seconds = static_cast<int32_t>(spec["scheduleTimeoutSeconds"].as_int());
  pg->phase = st["phase"].as_string();
  pg->occupied_by = st["occupiedBy"].as_string();
  pg->scheduled = static_cast<int32_t>(st["scheduled"].as_int(0));
  pg->running = static_cast<int32_t>(st["running"].as_int(0));
  pg->succeeded = static_cast<int32_t>(st["succeeded"].as_int(0));
  pg->failed = static_cast<int32_t>(st["failed"].as_int(0));
  if (st["scheduleStartTime"].is_string()) pg->schedule_start_time = parse_rfc3339(st["scheduleStartTime"].as_string());
  return pg;
}

std::shared_ptr<ElasticQuota> ElasticQuota::from_json(const Json& obj) {
  auto eq = std::make_shared<ElasticQuota>();
  eq->meta = ObjectMeta::from_json(obj);
  const Json& spec = obj["spec"];
  eq->has_min = spec.get("min") != nullptr;
  eq->has_max = spec.get("max") != nullptr;
  eq->min = Res::from_json(spec["min"]);
  eq->max = Res::from_json(spec["max"]);
  eq->used = Res::from_json(obj["status"]["used"]);
  return eq;
}

std::shared_ptr<NodeResourceTopology> NodeResourceTopology::from_json(const Json& obj) {
  auto nrt = std::make_shared<NodeResourceTopology>();
  nrt->meta = ObjectMeta::from_json(obj);
  for (const auto& p : obj["topologyPolicies"].items()) nrt->topology_policies.push_back(p.as_string());
  for (const auto& z : obj["zones"].items()) {
    NRTZone zone;
    zone.name = z["name"].as_string();
    zone.type = z["type"].as_string();
    if (zone.name.rfind("node-", 0) == 0) {
      char* e = nullptr;
      long id = std::strtol(zone.name.c_str() + 5, &e, 10);
      if (e && *e == '\0') zone.numa_id = static_cast<int>(id);
    }
    for (const auto& r : z["resources"].items()) {
      NRTResourceInfo ri;
      ri.name = r["name"].as_string();
      ri.res = res_id(ri.name);
      auto q = [&](const char* k) -> int64_t {
        const Json& v = r[k];
        if (v.is_string()) return quantity_to_res_units(ri.res, Quantity::parse(v.as_string()));
        if (v.is_number()) return quantity_to_res_units(ri.res, Quantity::from_int(v.as_int()));
        return 0;
      };
      ri.capacity = q("capacity");
      ri.allocatable = q("allocatable");
      ri.available = q("available");
      zone.resources.push_back(ri);
    }
    for (const auto& c : z["costs"].items()) zone.costs.emplace_back(c["name"].as_string(), c["value"].as_int());
    if (zone.type == "Node" && zone.numa_id >= 0 && zone.numa_id <= 63) {
      NumaZone nz;
      nz.id = zone.numa_id;
      for (const auto& r : zone.resources) nz.res.emplace_back(r.res, r.available);
      nrt->numa.push_back(std::move(nz));
    }
    nrt->zones.push_back(std::move(zone));
  }
  std::sort(nrt->numa.begin(), nrt->numa.end(), [](const NumaZone& a, const NumaZone& b) { return a.id < b.id; });
  return nrt;
}

std::shared_ptr<PodDisruptionBudget> PodDisruptionBudget::from_json(const Json& obj) {
  auto pdb = std::make_shared<PodDisruptionBudget>();
  pdb->meta = ObjectMeta::from_json(obj);
  pdb->selector = LabelSelector::from_json(obj["spec"].get("selector"));
  pdb->disruptions_allowed = static_cast<int32_t>(obj["status"]["disruptionsAllowed"].as_int(0));
  pdb->disrupted_pods = strmap_from_json(obj["status"]["disruptedPods"]);
  return pdb;
}

std::shared_ptr<PriorityClass> PriorityClass::from_json(const Json& obj) {
  auto pc = std::make_shared<PriorityClass>();
  pc->meta = ObjectMeta::from_json(obj);
  pc->value = static_cast<int32_t>(obj["value"].as_int(0));
  pc->global_default = obj["globalDefault"].as_bool(false);
  pc->preemption_policy = obj["preemptionPolicy"].as_string();
  return pc;
}

// ------------------------------------------------------------ GPU names ----
const GpuNames& default_gpu_names() {
  static const GpuNames* g = new GpuNames();
  return *g;
}
void GpuNames::intern() {
  gpu_rid_ = res_id(gpu);
  mem_rid_ = res_id(memory);
  xcd_rid_ = res_id(xcd);
}
std::shared_ptr<const GpuNames> GpuNames::from_args(const Json& args) {
  auto g = std::make_shared<GpuNames>();
  auto take = [&](const char* key, std::string& field) {
    if (args[key].is_string() && !args[key].as_string().empty()) field = args[key].as_string();
  };
  take("gpuResourceName", g->gpu);
  take("memoryResourceName", g->memory);
  take("xcdResourceName", g->xcd);
  take("indexAnnotationKey", g->index_annotation);
  take("partitionAnnotationKey", g->partition_annotation);
  g->intern();
  return g;
}
std::string GpuNames::describe() const {
  return "gpu=" + gpu + " memory=" + memory + " xcd=" + xcd + " index=" + index_annotation +
         " partitions=" + partition_annotation;
}

GpuDemand compute_gpu_demand(const Pod& p, const GpuNames& gn) {
  int gid = gn.gpu_id(), mid = gn.memory_id(), xid = gn.xcd_id();
  bool has_g = false, has_m = false, has_x = false;
  for (const auto& c : p.containers) {  // presence per container limit (podResourceLimit)
    has_g |= c.limits.has(gid);
    has_m |= c.limits.has(mid);
    has_x |= c.limits.has(xid);
  }
  GpuDemand d;
  int kinds = int(has_g) + int(has_m) + int(has_x);
  if (kinds == 0) return d;
  if (kinds > 1) {
    d.kind = GpuDemand::Conflict;
    return d;
  }
  if (has_g) {
    d.kind = GpuDemand::Gpu;
    d.amount = p.limit_sum().get(gid);
  } else if (has_x) {
    d.kind = GpuDemand::Xcd;
    d.amount = p.limit_sum().get(xid);
  } else {
    d.kind = GpuDemand::Memory;
    d.amount = p.limit_sum().get(mid);
  }
  return d;
}

}  // namespace xsched
