#include "scheduler/extender.h"

#include <cctype>
#include <stdexcept>

#include "api/resource.h"
#include "rest/kube.h"

namespace xsched {

namespace {

// Go's encoding/json matches object keys case-insensitively.
const Json* get_ci(const Json& obj, std::string_view key) {
  if (!obj.is_object()) return nullptr;
  if (const Json* v = obj.get(key)) return v;
  for (const auto& [k, v] : obj.members()) {
    if (k.size() != key.size()) continue;
    bool eq = true;
    for (size_t i = 0; i < k.size() && eq; ++i)
      eq = std::tolower(static_cast<unsigned char>(k[i])) == std::tolower(static_cast<unsigned char>(key[i]));
    if (eq) return &v;
  }
  return nullptr;
}

Json names_array(const std::vector<std::string>& nodes) {
  Json a = Json::array();
  for (const auto& n : nodes) a.push_back(Json(n));
  return a;
}

std::map<std::string, std::string> failed_map(const Json* j) {
  std::map<std::string, std::string> out;
  if (j && j->is_object())
    for (const auto& [k, v] : j->members()) out[k] = v.as_string();
  return out;
}

Json minimal_pod(const std::string& ns, const std::string& name, const std::string& uid) {
  Json md = Json::object();
  md.set("name", Json(name));
  md.set("namespace", Json(ns));
  if (!uid.empty()) md.set("uid", Json(uid));
  Json p = Json::object();
  p.set("apiVersion", Json("v1"));
  p.set("kind", Json("Pod"));
  p.set("metadata", std::move(md));
  return p;
}

}  // namespace

ExtenderConfig ExtenderConfig::from_json(const Json& j) {
  ExtenderConfig c;
  c.url_prefix = j["urlPrefix"].as_string();
  c.filter_verb = j["filterVerb"].as_string();
  c.prioritize_verb = j["prioritizeVerb"].as_string();
  c.bind_verb = j["bindVerb"].as_string();
  c.preempt_verb = j["preemptVerb"].as_string();
  c.weight = j["weight"].as_int(1);
  c.node_cache_capable = j["nodeCacheCapable"].as_bool(false);
  c.ignorable = j["ignorable"].as_bool(false);
  for (const auto& r : j["managedResources"].items()) c.managed_resources.insert(r["name"].as_string());
  // httpTimeout arrives in milliseconds from the Python loader (it accepts
  // Go durations such as "30s").
  int64_t t = j["httpTimeoutMs"].as_int(0);
  c.timeout_ms = t > 0 ? static_cast<int>(t) : 5000;
  c.enable_https = j["enableHTTPS"].as_bool(false);
  const Json& tls = j["tlsConfig"];
  c.tls.insecure = tls["insecure"].as_bool(false);
  c.tls.ca_file = tls["caFile"].as_string();
  c.tls.cert_file = tls["certFile"].as_string();
  c.tls.key_file = tls["keyFile"].as_string();
  c.tls.ca_pem = tls["caData"].as_string();
  c.tls.cert_pem = tls["certData"].as_string();
  c.tls.key_pem = tls["keyData"].as_string();
  return c;
}

Extender::Extender(ExtenderConfig c) : cfg_(std::move(c)) {
  // urlPrefix: scheme://host[:port][/path]
  std::string u = cfg_.url_prefix;
  bool https = false;
  if (u.rfind("https://", 0) == 0) {
    https = true;
    u = u.substr(8);
  } else if (u.rfind("http://", 0) == 0) {
    u = u.substr(7);
  } else {
    throw std::invalid_argument("extender urlPrefix must start with http:// or https://: " + cfg_.url_prefix);
  }
  size_t slash = u.find('/');
  std::string hostport = slash == std::string::npos ? u : u.substr(0, slash);
  path_prefix_ = slash == std::string::npos ? "" : u.substr(slash);
  while (!path_prefix_.empty() && path_prefix_.back() == '/') path_prefix_.pop_back();
  rest::Endpoint ep;
  size_t colon = hostport.rfind(':');
  if (!hostport.empty() && hostport.front() == '[') {  // [v6]:port
    size_t close = hostport.find(']');
    ep.host = hostport.substr(1, close - 1);
    colon = hostport.find(':', close);
  } else {
    ep.host = colon == std::string::npos ? hostport : hostport.substr(0, colon);
  }
  https = https || cfg_.enable_https;
  ep.port = colon == std::string::npos ? (https ? 443 : 80) : std::stoi(hostport.substr(colon + 1));
  ep.timeout_ms = cfg_.timeout_ms;
  if (https) {
    ep.tls = cfg_.tls;
    ep.tls.enabled = true;
    // extender.go makeTransport: enableHTTPS without a CA skips verification.
    if (ep.tls.ca_file.empty() && ep.tls.ca_pem.empty()) ep.tls.insecure = true;
  }
  pool_ = std::make_unique<rest::ConnPool>(ep);
}

Extender::~Extender() = default;

bool Extender::interested(const Pod& p) const {
  if (cfg_.managed_resources.empty()) return true;
  auto& reg = ResourceRegistry::get();
  for (const auto& name : cfg_.managed_resources) {
    int id = reg.find(name);
    if (id < 0) continue;
    for (const auto* cs : {&p.containers, &p.init_containers})
      for (const auto& c : *cs)
        if (c.requests.has(id) || c.limits.has(id)) return true;
  }
  return false;
}

Json Extender::send(const std::string& verb, const Json& args) {
  calls_.fetch_add(1, std::memory_order_relaxed);
  rest::Response r = pool_->call("POST", path_prefix_ + "/" + verb, args.dump());
  if (r.status != 200)
    throw std::runtime_error("extender " + cfg_.url_prefix + " " + verb + ": HTTP " + std::to_string(r.status) +
                             (r.body.empty() ? "" : ": " + r.body.substr(0, 200)));
  try {
    return r.body.empty() ? Json::object() : Json::parse(r.body);
  } catch (const std::exception& e) {
    throw std::runtime_error("extender " + cfg_.url_prefix + " " + verb + ": bad response: " + e.what());
  }
}

Json Extender::node_args(const Json& pod, const std::vector<std::string>& nodes, const ObjectLookup& lookup) const {
  Json args = Json::object();
  args.set("Pod", pod);
  if (cfg_.node_cache_capable) {
    args.set("NodeNames", names_array(nodes));
  } else {
    Json items = Json::array();
    for (const auto& n : nodes) {
      JsonPtr obj = lookup ? lookup("nodes", "", n) : nullptr;
      if (obj) {
        items.push_back(*obj);
      } else {
        Json md = Json::object();
        md.set("name", Json(n));
        Json o = Json::object();
        o.set("metadata", std::move(md));
        items.push_back(std::move(o));
      }
    }
    Json list = Json::object();
    list.set("apiVersion", Json("v1"));
    list.set("kind", Json("NodeList"));
    list.set("items", std::move(items));
    args.set("Nodes", std::move(list));
  }
  return args;
}

Extender::FilterResult Extender::filter(const Json& pod, const std::vector<std::string>& nodes,
                                        const ObjectLookup& lookup) {
  FilterResult out;
  if (!is_filter()) {
    out.nodes = nodes;
    return out;
  }
  Json res = send(cfg_.filter_verb, node_args(pod, nodes, lookup));
  if (const Json* e = get_ci(res, "Error"); e && !e->as_string().empty()) throw std::runtime_error(e->as_string());
  std::set<std::string> input(nodes.begin(), nodes.end());
  auto take = [&](const std::string& n) {
    if (!input.count(n))
      throw std::runtime_error("extender " + cfg_.url_prefix + " claims a filtered node " + n +
                               " which is not found in the input node list");
    out.nodes.push_back(n);
  };
  const Json* names = get_ci(res, "NodeNames");
  const Json* list = get_ci(res, "Nodes");
  if (cfg_.node_cache_capable && names && names->is_array()) {
    for (const auto& n : names->items()) take(n.as_string());
  } else if (list && list->is_object()) {
    for (const auto& n : (*get_ci(*list, "items")).items()) take(n["metadata"]["name"].as_string());
  } else if (names && names->is_array()) {  // a cache-less extender that answered with names
    for (const auto& n : names->items()) take(n.as_string());
  }
  out.failed = failed_map(get_ci(res, "FailedNodes"));
  out.unresolvable = failed_map(get_ci(res, "FailedAndUnresolvableNodes"));
  return out;
}

std::vector<std::pair<std::string, int64_t>> Extender::prioritize(const Json& pod, const std::vector<std::string>& nodes,
                                                                  const ObjectLookup& lookup) {
  std::vector<std::pair<std::string, int64_t>> out;
  if (!is_prioritizer()) return out;
  Json res = send(cfg_.prioritize_verb, node_args(pod, nodes, lookup));
  for (const auto& hp : res.items()) {
    const Json* h = get_ci(hp, "Host");
    const Json* s = get_ci(hp, "Score");
    if (h && s) out.emplace_back(h->as_string(), s->as_int());
  }
  return out;
}

void Extender::bind(const std::string& ns, const std::string& name, const std::string& uid, const std::string& node) {
  Json args = Json::object();
  args.set("PodName", Json(name));
  args.set("PodNamespace", Json(ns));
  args.set("PodUID", Json(uid));
  args.set("Node", Json(node));
  Json res = send(cfg_.bind_verb, args);
  if (const Json* e = get_ci(res, "Error"); e && !e->as_string().empty()) throw std::runtime_error(e->as_string());
}

std::map<std::string, Extender::NodeVictims> Extender::process_preemption(
    const Json& pod, const std::map<std::string, NodeVictims>& in, const ObjectLookup& lookup) {
  Json args = Json::object();
  args.set("Pod", pod);
  Json victims = Json::object();
  for (const auto& [node, v] : in) {
    Json pods = Json::array();
    for (const auto& p : v.pods) {
      if (cfg_.node_cache_capable) {
        Json mp = Json::object();
        mp.set("UID", Json(p->uid()));
        pods.push_back(std::move(mp));
      } else {
        JsonPtr obj = lookup ? lookup("pods", p->ns(), p->name()) : nullptr;
        pods.push_back(obj ? *obj : minimal_pod(p->ns(), p->name(), p->uid()));
      }
    }
    Json e = Json::object();
    e.set("Pods", std::move(pods));
    e.set("NumPDBViolations", Json(v.num_pdb_violations));
    victims.set(node, std::move(e));
  }
  args.set(cfg_.node_cache_capable ? "NodeNameToMetaVictims" : "NodeNameToVictims", std::move(victims));
  Json res = send(cfg_.preempt_verb, args);
  // The extender always answers with meta victims (UIDs), which must name
  // pods of the offered candidates (extender.go convertPodUIDToPod).
  std::map<std::string, NodeVictims> out;
  const Json* m = get_ci(res, "NodeNameToMetaVictims");
  if (!m || !m->is_object()) return out;
  for (const auto& [node, mv] : m->members()) {
    auto it = in.find(node);
    if (it == in.end()) throw std::runtime_error("extender " + cfg_.url_prefix + " returned unknown node " + node);
    NodeVictims nv;
    const Json* pods = get_ci(mv, "Pods");
    if (pods)
      for (const auto& mp : pods->items()) {
        const Json* uid = get_ci(mp, "UID");
        std::string u = uid ? uid->as_string() : "";
        PodPtr found;
        for (const auto& p : it->second.pods)
          if (p->uid() == u) found = p;
        if (!found)
          throw std::runtime_error("extender: " + cfg_.url_prefix + " claims to preempt pod (UID: " + u +
                                   ") on node: " + node + ", but the pod is not found on that node");
        nv.pods.push_back(found);
      }
    if (const Json* pv = get_ci(mv, "NumPDBViolations")) nv.num_pdb_violations = pv->as_int();
    out[node] = std::move(nv);
  }
  return out;
}

}  // namespace xsched
