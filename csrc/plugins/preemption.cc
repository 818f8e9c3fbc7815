// DefaultPreemption and PreemptionToleration (PostFilter plugins on the
// shared Evaluator, scheduler/preemption.h).
//
// PreemptionToleration reference: pkg/preemptiontoleration/
// preemption_toleration.go:102-315 and preemption_toleration_policy.go:25-82.
// A victim candidate (lower priority than the preemptor) is exempt iff its
// PriorityClass parses and: the preemptor's policy is Never, or preemptor
// priority < minimum-preemptable-priority (default PC.value+1) and
// (toleration-seconds < 0, or the victim is not scheduled yet, or it was
// scheduled less than toleration-seconds ago).
#include <cerrno>
#include <cstdlib>
#include <random>

#include "framework/plugin.h"
#include "scheduler/informers.h"
#include "scheduler/preemption.h"

namespace xsched {
namespace {

inline constexpr const char* kAnnMinPreemptable = "preemption-toleration.scheduling.sigs.k8s.io/minimum-preemptable-priority";
inline constexpr const char* kAnnTolerationSeconds = "preemption-toleration.scheduling.sigs.k8s.io/toleration-seconds";

class DefaultPreemption : public Plugin, public PreemptionPolicy {
 public:
  DefaultPreemption(const Json& args, Handle& h, std::string name = "DefaultPreemption")
      : Plugin(std::move(name), kPostFilter), h_(h), ev_(name_, h, this) {
    pct_ = static_cast<int>(args["minCandidateNodesPercentage"].as_int(10));
    abs_ = static_cast<int>(args["minCandidateNodesAbsolute"].as_int(100));
    rng_.seed(static_cast<uint64_t>(wall_now_us()));
  }

  std::pair<PostFilterResult, Status> post_filter(CycleState& s, const Pod& p, const NodeStatusMap& m) override {
    return ev_.preempt(s, p, m);
  }

  std::pair<int, int> offset_and_num_candidates(int n) override {
    std::lock_guard<std::mutex> g(rng_mu_);
    int off = n > 0 ? static_cast<int>(rng_() % static_cast<uint64_t>(n)) : 0;
    return {off, calculate_num_candidates(n, pct_, abs_)};
  }
  bool eligible(const Pod& pod, const Status* nom) override { return default_eligible(h_, pod, nom); }
  Status select_victims_on_node(CycleState& s, const Pod& preemptor, NodeInfo& ni, const std::vector<PDBPtr>& pdbs,
                                std::vector<PodPtr>& victims, int& num_violating) override {
    int32_t prio = preemptor.priority;
    return select_victims_default(h_, s, preemptor, ni, pdbs, [&](const Pod& p) { return p.priority < prio; }, victims,
                                 num_violating);
  }
  // Victims = lower-priority pods, kept or reprieved by node-local Filters:
  // a function of the node and the preemptor alone. Subclasses with their
  // own victim rules (PreemptionToleration: clock-dependent) opt out.
  bool victims_depend_only_on_node() const override { return !overrides_victims_; }
  // Default and PreemptionToleration victims are lower-priority pods (the
  // latter only narrows that set).
  bool victims_have_lower_priority() const override { return true; }

 protected:
  bool overrides_victims_ = false;  // set by subclasses that replace select_victims_on_node
  Handle& h_;
  Evaluator ev_;
  int pct_ = 10, abs_ = 100;
  std::mutex rng_mu_;
  std::mt19937_64 rng_;
};

struct TolerationPolicy {
  int32_t min_preemptable = 0;
  int64_t toleration_seconds = 0;
};

// parsePreemptionTolerationPolicy (preemption_toleration_policy.go:54-82);
// `err` (optional) receives Go's strconv.ParseInt message on failure.
bool parse_policy(const PriorityClass& pc, TolerationPolicy* out, std::string* err = nullptr) {
  out->min_preemptable = pc.value + 1;
  out->toleration_seconds = 0;
  auto parse = [&](const std::string& v, int bits, long long* x) {
    char* e = nullptr;
    errno = 0;
    *x = std::strtoll(v.c_str(), &e, 10);
    const bool range = errno == ERANGE || (bits == 32 && (*x < INT32_MIN || *x > INT32_MAX));
    if (!v.empty() && !*e && !range) return true;
    if (err) *err = "strconv.ParseInt: parsing \"" + v + "\": " + (range && !*e ? "value out of range" : "invalid syntax");
    return false;
  };
  long long x = 0;
  if (const std::string* v = pc.meta.annotation(kAnnMinPreemptable)) {
    if (!parse(*v, 32, &x)) return false;
    out->min_preemptable = static_cast<int32_t>(x);
  }
  if (const std::string* v = pc.meta.annotation(kAnnTolerationSeconds)) {
    if (!parse(*v, 64, &x)) return false;
    out->toleration_seconds = x;
  }
  return true;
}

class PreemptionToleration : public DefaultPreemption {
 public:
  PreemptionToleration(const Json& args, Handle& h) : DefaultPreemption(args, h, "PreemptionToleration") {
    overrides_victims_ = true;
  }

  // ExemptedFromPreemption (preemption_toleration.go:125-175). `err`
  // (optional) receives the lister's not-found error the reference returns.
  bool exempted(const Pod& victim, const Pod& preemptor, MicroTime now, std::string* err = nullptr) const {
    if (victim.priority_class_name.empty()) return false;
    auto pc = h_.informers->priority_class(victim.priority_class_name);
    if (!pc) {  // lister miss: no toleration (the reference surfaces the error)
      if (err) *err = "priorityclass.scheduling.k8s.io \"" + victim.priority_class_name + "\" not found";
      return false;
    }
    if (preemptor.preemption_policy == "Never") return true;
    TolerationPolicy pol;
    if (!parse_policy(*pc, &pol)) return false;
    if (preemptor.priority >= pol.min_preemptable) return false;
    if (pol.toleration_seconds < 0) return true;
    if (victim.scheduled_at == 0) return true;
    return victim.scheduled_at + pol.toleration_seconds * 1000000 > now;
  }

  // Unit-test hooks for preemption_toleration_test.go (exemptedFromPreemption:
  // args.victim, args.preemptor, args.nowUs) and
  // preemption_toleration_policy_test.go (parsePolicy: args.priorityClass).
  Json debug_call(const std::string& what, CycleState& s, const PodPtr& p, const Json& args) override {
    Json out = Json::object();
    if (what == "exemptedFromPreemption") {
      auto victim = Pod::from_json(args["victim"], *h_.gpu_names);
      auto preemptor = Pod::from_json(args["preemptor"], *h_.gpu_names);
      std::string err;
      const bool ex = exempted(*victim, *preemptor, args["nowUs"].as_int(wall_now_us()), &err);
      if (!err.empty()) out.set("error", Json(err));
      else out.set("exempted", Json(ex));
      return out;
    }
    if (what == "parsePolicy") {
      auto pc = PriorityClass::from_json(args["priorityClass"]);
      TolerationPolicy pol;
      std::string err;
      if (!parse_policy(*pc, &pol, &err)) {
        out.set("error", Json(err));
      } else {
        out.set("minimumPreemptablePriority", Json(static_cast<int64_t>(pol.min_preemptable)));
        out.set("tolerationSeconds", Json(static_cast<int64_t>(pol.toleration_seconds)));
      }
      return out;
    }
    return Plugin::debug_call(what, s, p, args);
  }

  Status select_victims_on_node(CycleState& s, const Pod& preemptor, NodeInfo& ni, const std::vector<PDBPtr>& pdbs,
                                std::vector<PodPtr>& victims, int& num_violating) override {
    int32_t prio = preemptor.priority;
    MicroTime now = wall_now_us();
    return select_victims_default(
        h_, s, preemptor, ni, pdbs, [&](const Pod& p) { return p.priority < prio && !exempted(p, preemptor, now); },
        victims, num_violating);
  }
};

PluginRegistrar r1("DefaultPreemption", [](const Json& a, Handle& h) { return std::make_shared<DefaultPreemption>(a, h); });
PluginRegistrar r2("PreemptionToleration",
                   [](const Json& a, Handle& h) { return std::make_shared<PreemptionToleration>(a, h); });

}  // namespace

void link_preemption_plugins() {}

}  // namespace xsched
