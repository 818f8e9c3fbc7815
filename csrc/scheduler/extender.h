// HTTP scheduler extenders: the `extenders:` block of a
// KubeSchedulerConfiguration.
//
// Reference: vendor/k8s.io/kubernetes/pkg/scheduler/extender.go:148-409
// (HTTPExtender: Filter / Prioritize / Bind / ProcessPreemption, IsInterested
// over managedResources, ignorable, nodeCacheCapable), wired into the cycle at
// generic_scheduler.go:193-212,258 (findNodesThatPassExtenders after the
// Filter plugins, also for the nominated node), :449-488 (extender scores x
// weight x MaxNodeScore/MaxExtenderPriority added to the plugin totals),
// scheduler.go bind() (the first interested binder extender binds instead of
// the Bind plugins) and preemption.go callExtenders (candidates filtered by
// the preempt verb).
//
// The wire format is kube-scheduler/extender/v1 marshalled by encoding/json
// without tags: Go field names ("Pod", "Nodes", "NodeNames", "FailedNodes",
// "NodeNameToVictims", ...). Responses are read case-insensitively, as Go's
// decoder does.
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "api/types.h"
#include "common/json.h"
#include "rest/http.h"

namespace xsched {

namespace rest {
class ConnPool;
}

inline constexpr int64_t kMaxExtenderPriority = 10;

struct ExtenderConfig {
  std::string url_prefix;
  std::string filter_verb, prioritize_verb, bind_verb, preempt_verb;
  int64_t weight = 1;
  bool node_cache_capable = false;
  bool ignorable = false;
  std::set<std::string> managed_resources;
  int timeout_ms = 5000;  // DefaultExtenderTimeout
  bool enable_https = false;
  rest::TlsOptions tls;
  // Decodes one entry of the config's extenders list (the Python loader has
  // validated and defaulted it: config.py _extenders).
  static ExtenderConfig from_json(const Json& j);
};

// Looks up the API object of a kind/ns/name (the informer store): extenders
// receive whole Pod and Node objects unless they are nodeCacheCapable.
using ObjectLookup = std::function<JsonPtr(const std::string& kind, const std::string& ns, const std::string& name)>;

class Extender {
 public:
  explicit Extender(ExtenderConfig c);
  ~Extender();
  const std::string& name() const { return cfg_.url_prefix; }
  const ExtenderConfig& config() const { return cfg_; }
  bool ignorable() const { return cfg_.ignorable; }
  bool is_binder() const { return !cfg_.bind_verb.empty(); }
  bool is_filter() const { return !cfg_.filter_verb.empty(); }
  bool is_prioritizer() const { return !cfg_.prioritize_verb.empty(); }
  bool supports_preemption() const { return !cfg_.preempt_verb.empty(); }
  // True when managedResources is empty or any (init) container requests or
  // limits one of them.
  bool interested(const Pod& p) const;

  struct FilterResult {
    std::vector<std::string> nodes;              // nodes that pass (subset of the input)
    std::map<std::string, std::string> failed;   // -> Unschedulable
    std::map<std::string, std::string> unresolvable;  // -> UnschedulableAndUnresolvable
  };
  // Throws std::runtime_error on transport errors, an Error in the result or
  // a node outside the input list.
  FilterResult filter(const Json& pod, const std::vector<std::string>& nodes, const ObjectLookup& lookup);
  // (host, score in [0, 10]) pairs; the caller multiplies by weight.
  std::vector<std::pair<std::string, int64_t>> prioritize(const Json& pod, const std::vector<std::string>& nodes,
                                                          const ObjectLookup& lookup);
  void bind(const std::string& ns, const std::string& name, const std::string& uid, const std::string& node);
  // node -> victims the extender accepts (it answers with UIDs, which must
  // name offered victims of that node); nodes it drops are absent.
  struct NodeVictims {
    std::vector<PodPtr> pods;
    int64_t num_pdb_violations = 0;
  };
  std::map<std::string, NodeVictims> process_preemption(const Json& pod, const std::map<std::string, NodeVictims>& in,
                                                        const ObjectLookup& lookup);

  uint64_t calls() const { return calls_; }

 private:
  Json send(const std::string& verb, const Json& args);
  Json node_args(const Json& pod, const std::vector<std::string>& nodes, const ObjectLookup& lookup) const;

  ExtenderConfig cfg_;
  std::string path_prefix_;  // path part of urlPrefix, without the trailing '/'
  std::unique_ptr<rest::ConnPool> pool_;
  std::atomic<uint64_t> calls_{0};
};

using ExtenderList = std::vector<std::shared_ptr<Extender>>;

}  // namespace xsched
