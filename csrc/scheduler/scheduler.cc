#include "scheduler/scheduler.h"

#include "common/log.h"
#include "common/reaper.h"

#include <algorithm>
#include <cstring>
#include <optional>
#include <chrono>
#include <thread>
#include <map>
#include <stdexcept>

namespace xsched {

// ----------------------------------------------------------- StoreClient ----
void StoreClient::bind(const Pod& pod, const std::string& node, const Json& annotations) {
  store_->bind(pod.ns(), pod.name(), pod.uid(), node, annotations);
}

void StoreClient::delete_pod(const Pod& pod) { store_->remove("pods", pod.ns(), pod.name(), 0, pod.uid()); }

void StoreClient::patch(const std::string& kind, const std::string& ns, const std::string& name, const Json& patch) {
  store_->patch(kind, ns, name, patch);
}

void StoreClient::record_event(const std::string& kind, const std::string& ns, const std::string& name,
                               const std::string& type, const std::string& reason, const std::string& msg) {
  if (!events_enabled) return;
  const int64_t now = wall_now_us();
  std::string corr;
  corr.reserve(kind.size() + ns.size() + name.size() + reason.size() + msg.size() + 4);
  corr.append(kind).push_back('\0');
  corr.append(ns).push_back('\0');
  corr.append(name).push_back('\0');
  corr.append(reason).push_back('\0');
  corr.append(msg);
  Recent seen;
  {
    std::lock_guard<std::mutex> g(events_mu_);
    auto it = recent_.find(corr);
    if (it != recent_.end() && now - it->second.last_us < kAggregateUs) {
      it->second.count += 1;
      it->second.last_us = now;
      seen = it->second;
    }
  }
  if (seen.count > 0) {
    Json p = Json::object();
    p.set("count", Json(seen.count));
    p.set("lastTimestamp", Json(format_rfc3339(now)));
    try {
      store_->patch("events", seen.ns, seen.name, p);
      return;
    } catch (const StoreError&) {
      // expired or deleted: record a fresh Event below
    }
  }
  Json ev = Json::object();
  Json md = Json::object();
  md.set("generateName", Json(name + "."));
  md.set("namespace", Json(ns.empty() ? "default" : ns));
  ev.set("metadata", std::move(md));
  Json ref = Json::object();
  ref.set("kind", Json(kind));
  ref.set("namespace", Json(ns));
  ref.set("name", Json(name));
  ev.set("involvedObject", std::move(ref));
  ev.set("type", Json(type));
  ev.set("reason", Json(reason));
  ev.set("message", Json(msg));
  ev.set("reportingController", Json("xsched"));
  ev.set("count", Json(int64_t{1}));
  ev.set("firstTimestamp", Json(format_rfc3339(now)));
  ev.set("lastTimestamp", Json(format_rfc3339(now)));
  JsonPtr created;
  try {
    created = store_->create("events", std::move(ev));
  } catch (const StoreError&) {
    return;
  }
  const Json& md2 = (*created)["metadata"];
  std::lock_guard<std::mutex> g(events_mu_);
  recent_[std::move(corr)] = Recent{md2["namespace"].as_string(), md2["name"].as_string(), 1, now};
  if (recent_.size() > recent_sweep_at_) {  // amortized: sweep when doubled
    for (auto it = recent_.begin(); it != recent_.end();)
      it = now - it->second.last_us >= kAggregateUs ? recent_.erase(it) : std::next(it);
    recent_sweep_at_ = std::max<size_t>(4096, 2 * recent_.size());
  }
}

// -------------------------------------------------------------- Executor ----
bool Executor::try_pop(std::function<void()>& fn) {
  if (q_.empty()) return false;
  fn = std::move(q_.front());
  q_.pop_front();
  queued_.fetch_sub(1, std::memory_order_relaxed);
  busy_.fetch_add(1);
  return true;
}

Executor::Executor(int threads) {
  if (const char* e = std::getenv("XSCHED_BIND_SPIN_NS")) spin_ns_ = std::max<int64_t>(0, std::atoll(e));
  base_ = std::max(1, threads);
  std::lock_guard<AdaptiveMutex> g(mu_);
  for (int i = 0; i < base_; ++i) spawn_locked();
}

void Executor::spawn_locked() {
  threads_.emplace_back([this] {
    name_this_thread("xs-bind");
    bool spin = false;  // just finished a task: poll before sleeping
    for (;;) {
      std::function<void()> fn;
      if (spin && spin_ns_ > 0) {
        if (spinners_.fetch_add(1) < kMaxSpinners) {
          const int64_t until = Parallelizer::now_ns() + spin_ns_;
          while (queued_.load(std::memory_order_relaxed) == 0 && Parallelizer::now_ns() < until)
            __builtin_ia32_pause();
        }
        // Leave the spinner set before the locked check below: a submit
        // that still saw this spinner finds its task taken here.
        spinners_.fetch_sub(1);
      }
      bool chain = false;
      {
        std::unique_lock<AdaptiveMutex> lk(mu_);
        if (!try_pop(fn)) {
          ++waiters_;
          while (!stop_ && q_.empty()) {
            cv_.wait(lk);
            if (wakes_ > 0) --wakes_;  // every wake-up consumes one, taken task or not
          }
          --waiters_;
          if (!try_pop(fn)) return;  // stop_ and drained
        }
        // Chain wake-up: a burst submitted at once (a gang's Allows) costs
        // the submitter one futex wake; each woken worker wakes the next.
        if (!q_.empty() && waiters_ > 0 && wakes_ == 0 && queued_.load(std::memory_order_relaxed) > spinners_.load()) {
          ++wakes_;
          chain = true;
        }
      }
      if (chain) cv_.notify_one();
      fn();
      busy_.fetch_sub(1);
      spin = true;
    }
  });
}

void Executor::enter_blocking() {
  std::lock_guard<AdaptiveMutex> g(mu_);
  ++blocked_;
  // Keep `base_` workers able to run tasks (Go's runtime hands a P to a new
  // M when a goroutine blocks in a syscall): the pool grows to the
  // high-water mark of concurrently blocked tasks, capped.
  if (!stop_ && static_cast<int>(threads_.size()) - blocked_ < base_ && threads_.size() < kMaxThreads) spawn_locked();
}

void Executor::exit_blocking() {
  std::lock_guard<AdaptiveMutex> g(mu_);
  --blocked_;
}

size_t Executor::threads() const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  return threads_.size();
}

Executor::~Executor() { stop(); }

namespace {
thread_local Executor::Batch* tl_batch = nullptr;
}  // namespace

Executor::Batch::Batch(Executor& e) : e_(e), prev_(tl_batch) { tl_batch = this; }

Executor::Batch::~Batch() {
  tl_batch = prev_;
  if (fns_.empty()) return;
  bool wake = false;
  {
    std::lock_guard<AdaptiveMutex> g(e_.mu_);
    for (auto& fn : fns_) e_.q_.push_back(std::move(fn));
    e_.queued_.fetch_add(static_cast<int>(fns_.size()), std::memory_order_relaxed);
    if (e_.waiters_ > 0 && e_.wakes_ == 0 && e_.queued_.load(std::memory_order_relaxed) > e_.spinners_.load()) {
      ++e_.wakes_;
      wake = true;
    }
  }
  if (wake) e_.cv_.notify_one();
}

void Executor::submit(std::function<void()> fn) {
  for (Batch* b = tl_batch; b; b = b->prev_)
    if (&b->e_ == this) {
      b->fns_.push_back(std::move(fn));
      return;
    }
  bool wake = false;
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    q_.push_back(std::move(fn));
    queued_.fetch_add(1, std::memory_order_relaxed);
    // Wake a sleeper unless a spinning worker is free for this task or a
    // wake-up is already on its way (that worker wakes the next one).
    if (waiters_ > 0 && wakes_ == 0 && queued_.load(std::memory_order_relaxed) > spinners_.load()) {
      ++wakes_;
      wake = true;
    }
  }
  if (wake) cv_.notify_one();
}

void Executor::stop() {
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    if (stop_) return;
    stop_ = true;
  }
  cv_.notify_all();
  std::vector<std::thread> ts;
  {
    std::lock_guard<AdaptiveMutex> g(mu_);
    ts.swap(threads_);  // no spawn after stop_
  }
  for (auto& t : ts) t.join();
}

size_t Executor::pending() const {
  std::lock_guard<AdaptiveMutex> g(mu_);
  return q_.size() + static_cast<size_t>(busy_.load());
}

// ------------------------------------------------------- SchedulerOptions ----
SchedulerOptions SchedulerOptions::from_json(const Json& j) {
  SchedulerOptions o;
  o.parallelism = static_cast<int>(j["parallelism"].as_int(o.parallelism));
  o.bind_workers = static_cast<int>(j["bindWorkers"].as_int(o.bind_workers));
  o.parallel_inline_below = static_cast<int>(j["parallelInlineBelow"].as_int(o.parallel_inline_below));
  o.percentage_of_nodes_to_score = static_cast<int>(j["percentageOfNodesToScore"].as_int(0));
  if (j["podInitialBackoffSeconds"].is_number())
    o.pod_initial_backoff_us = static_cast<int64_t>(j["podInitialBackoffSeconds"].as_double() * 1e6);
  if (j["podMaxBackoffSeconds"].is_number())
    o.pod_max_backoff_us = static_cast<int64_t>(j["podMaxBackoffSeconds"].as_double() * 1e6);
  if (j["assumedPodTTLSeconds"].is_number())
    o.assumed_pod_ttl_us = static_cast<int64_t>(j["assumedPodTTLSeconds"].as_double() * 1e6);
  o.metrics_sample_rate = j["metricsSampleRate"].as_double(o.metrics_sample_rate);
  o.status_updates = j["statusUpdates"].as_bool(o.status_updates);
  o.events = j["events"].as_bool(o.events);
  o.equivalence_cache = j["equivalenceCache"].as_bool(o.equivalence_cache);
  auto env_on = [](const char* var) {
    const char* v = std::getenv(var);
    return !v || std::string(v) != "0";
  };
  o.gang_window = j["gangWindow"].as_bool(env_on("XSCHED_GANG_WINDOW"));
  o.scan_memo = j["scanMemo"].as_bool(env_on("XSCHED_SCAN_MEMO"));
  o.scan_memo_verify = j["scanMemoVerify"].as_bool(false);
  o.trace = j["trace"].as_bool(false);
  o.seed = static_cast<uint64_t>(j["seed"].as_int(0));
  o.dump_on_fit_error = j["dumpOnFitError"].str_or("");
  o.gang_denial_census = j["gangDenialCensus"].as_bool(false);
  return o;
}

// ------------------------------------------------------------- Scheduler ----
namespace {
const std::vector<std::string> kBaseKinds = {"pods", "nodes", "podgroups", "elasticquotas", "noderesourcetopologies",
                                             "poddisruptionbudgets", "priorityclasses"};
std::string resource_for_kind(const std::string& kind) {
  if (kind == "pods") return "Pod";
  if (kind == "nodes") return "Node";
  if (kind == "podgroups") return "PodGroup";
  if (kind == "elasticquotas") return "ElasticQuota";
  if (kind == "noderesourcetopologies") return "NodeResourceTopology";
  if (kind == "poddisruptionbudgets") return "PodDisruptionBudget";
  if (kind == "priorityclasses") return "PriorityClass";
  if (kind == "persistentvolumes") return "PersistentVolume";
  if (kind == "persistentvolumeclaims") return "PersistentVolumeClaim";
  if (kind == "storageclasses") return "StorageClass";
  if (kind == "csinodes") return "CSINode";
  return kind;
}
uint32_t action_for(EventType t) {
  switch (t) {
    case EventType::Added: return kAdd;
    case EventType::Deleted: return kDelete;
    default: return kUpdate;
  }
}
}  // namespace

Scheduler::Scheduler(std::shared_ptr<ObjectStore> store, const Json& config, std::shared_ptr<Clock> clock,
                     std::shared_ptr<ApiClient> client)
    : store_(std::move(store)), clock_(clock ? std::move(clock) : std::make_shared<RealClock>()) {
  register_builtin_plugins();
  opts_ = SchedulerOptions::from_json(config["options"]);
  rng_.seed(opts_.seed ? opts_.seed : static_cast<uint64_t>(clock_->now_us()));
  tracer_.enable(opts_.trace);
  timers_ = std::make_unique<TimerService>(clock_);
  parallelizer_ = std::make_unique<Parallelizer>(opts_.parallelism, opts_.parallel_inline_below);
  if (const char* v = std::getenv("XSCHED_INFORMER_WINDOW")) informer_window_ = std::max<size_t>(1, std::atoll(v));
  // XSCHED_PARSE_POOL=1: parse informer windows on 4 helper threads. Off by
  // default: on the 16-CPU L3 domain a shard runs in, the helpers' spinning
  // made some box runs markedly slower (profiles/r4q_treeab_*).
  if (const char* v = std::getenv("XSCHED_PARSE_POOL"); v && std::string(v) == "1")
    parse_pool_ = std::make_unique<Parallelizer>(4, 32, "xs-parse");
  metrics_ = std::make_unique<Metrics>();
  cache_ = std::make_unique<SchedulerCache>(clock_, opts_.assumed_pod_ttl_us);
  informers_ = std::make_unique<Informers>();
  nominator_ = std::make_unique<Nominator>();
  if (client) {
    client_ = std::move(client);
  } else {
    auto sc = std::make_shared<StoreClient>(store_);
    sc->events_enabled = opts_.events;
    client_ = std::move(sc);
  }

  for (const auto& ej : config["extenders"].items())
    extenders_.push_back(std::make_shared<Extender>(ExtenderConfig::from_json(ej)));
  const auto& profiles = config["profiles"].items();
  if (profiles.empty()) throw std::runtime_error("scheduler config has no profiles");
  // GPU names: every profile's FlexGPU args must agree (one cache, one GPU
  // ledger per node); other schedulers in the process are unaffected.
  for (const auto& pj : profiles) {
    const Json* args = pj["pluginConfig"].get("FlexGPU");
    if (!args) continue;
    auto gn = GpuNames::from_args(*args);
    if (!gpu_names_) gpu_names_ = gn;
    else if (!(*gn == *gpu_names_))
      throw std::runtime_error("FlexGPU resource names differ between profiles of one scheduler (" +
                               gpu_names_->describe() + " vs " + gn->describe() + ")");
  }
  if (!gpu_names_) gpu_names_ = std::make_shared<GpuNames>();
  cache_->set_gpu_names(gpu_names_.get());
  for (const auto& pj : profiles) {
    ProfileConfig pc = ProfileConfig::from_json(pj);
    if (pc.percentage_of_nodes_to_score == 0) pc.percentage_of_nodes_to_score = opts_.percentage_of_nodes_to_score;
    if (by_name_.count(pc.scheduler_name)) throw std::runtime_error("duplicate profile " + pc.scheduler_name);
    waiting_.push_back(std::make_unique<WaitingPods>(timers_.get()));
    Handle h;
    h.cache = cache_.get();
    h.informers = informers_.get();
    h.client = client_.get();
    h.waiting_pods = waiting_.back().get();
    h.parallelizer = parallelizer_.get();
    h.nominator = nominator_.get();
    h.clock = clock_;
    h.timers = timers_.get();
    h.activate = [this](const std::vector<PodPtr>& pods) { queue_->activate(pods); };
    h.deactivate = [this](const std::vector<PodPtr>& pods) { queue_->deactivate(pods); };
    h.gang_denied = [this](const Pod& p, const char* why) { note_gang_denied(p, why); };
    h.gang_parked = [this](const Pod&) { gang_parks_total_.fetch_add(1, std::memory_order_relaxed); };
    gang_placements_.push_back(std::make_unique<GangPlacement>(cache_.get(), clock_));
    h.gangs = gang_placements_.back().get();
    h.gang_planned = [this](const Pod& p, bool hostable) { note_gang_planned(p, hostable); };
    h.blocking_begin = [this] {
      if (binder_) binder_->enter_blocking();
    };
    h.blocking_end = [this] {
      if (binder_) binder_->exit_blocking();
    };
    h.metrics = metrics_.get();
    h.snapshot = &snapshot_;
    h.extenders = &extenders_;
    h.gpu_names = gpu_names_.get();
    h.lookup = [this](const std::string& kind, const std::string& ns, const std::string& name) {
      return store_->get(kind, ns, name);
    };
    frameworks_.push_back(std::make_unique<Framework>(pc, h));
    by_name_[pc.scheduler_name] = frameworks_.back().get();
  }
  // All profiles must share the queue sort (k8s validation); use the first.
  Framework* first = frameworks_.front().get();
  QueueOptions qo;
  qo.initial_backoff_us = opts_.pod_initial_backoff_us;
  qo.max_backoff_us = opts_.pod_max_backoff_us;
  queue_ = std::make_unique<SchedulingQueue>(
      [first](const QueuedPodInfo& a, const QueuedPodInfo& b) { return first->less(a, b); }, clock_, qo,
      nominator_.get());
  std::vector<std::pair<ClusterEvent, std::set<std::string>>> emap;
  for (const auto& fw : frameworks_) {
    for (const auto& pl : fw->all_plugins()) {
      for (const auto& ev : pl->events_to_register()) {
        bool merged = false;
        for (auto& [e, names] : emap)
          if (e.resource == ev.resource && e.action == ev.action) {
            names.insert(pl->name());
            merged = true;
          }
        if (!merged) emap.push_back({ev, {pl->name()}});
      }
    }
    for (const auto& k : fw->watched_kinds())
      if (std::find(plugin_kinds_.begin(), plugin_kinds_.end(), k) == plugin_kinds_.end()) plugin_kinds_.push_back(k);
  }
  queue_->set_cluster_event_map(std::move(emap));
  binder_ = std::make_unique<Executor>(opts_.bind_workers);
  status_writer_ = std::make_unique<Executor>(1);

  std::set<std::string> kinds(kBaseKinds.begin(), kBaseKinds.end());
  for (const auto& k : plugin_kinds_) kinds.insert(k);
  // Initial LIST (as informers do) then WATCH from that version.
  int64_t rv = 0;
  std::vector<WatchEvent> initial;
  for (const auto& k : kinds) {
    for (const auto& obj : store_->list(k, "", &rv)) initial.push_back(WatchEvent{EventType::Added, k, obj, nullptr, 0});
  }
  // Nodes before pods so assigned pods land on real NodeInfos.
  std::stable_sort(initial.begin(), initial.end(), [](const WatchEvent& a, const WatchEvent& b) {
    auto rank = [](const std::string& k) { return k == "nodes" ? 0 : k == "pods" ? 2 : 1; };
    return rank(a.kind) < rank(b.kind);
  });
  watcher_ = store_->watch(kinds, "", 0);
  // Events committed between list() and watch() would be lost: re-list is
  // avoided by watching from the listed version when history allows.
  store_->unwatch(watcher_);
  watcher_ = store_->watch(kinds, "", rv);
  for (const auto& ev : initial) handle_event(ev);
}

Scheduler::~Scheduler() { stop(); }

void Scheduler::start() {
  if (running_.exchange(true)) return;
  for (auto& fw : frameworks_) fw->start();
  // Backoff expiry is checked every 100 ms (upstream: 1 s), so a retried
  // pod waits its backoff, not its backoff plus up to a second of tick phase.
  timer_ids_.push_back(timers_->every(100'000, [this] { queue_->flush_backoff_completed(); }));
  timer_ids_.push_back(timers_->every(30'000'000, [this] { queue_->flush_unschedulable_leftover(); }));
  timer_ids_.push_back(timers_->every(1'000'000, [this] { cache_->cleanup_expired_assumed_pods(); }));
  timer_ids_.push_back(timers_->every(1'000'000, [this] {
    auto c = queue_->counts();
    metrics_->set_gauge("scheduler_pending_pods", "queue=\"active\"", static_cast<double>(c.active));
    metrics_->set_gauge("scheduler_pending_pods", "queue=\"backoff\"", static_cast<double>(c.backoff));
    metrics_->set_gauge("scheduler_pending_pods", "queue=\"unschedulable\"", static_cast<double>(c.unschedulable));
    metrics_->set_gauge("scheduler_pending_pods", "queue=\"parked\"", static_cast<double>(c.parked));
    // Upstream metrics.go:102 (Goroutines, by work) and :171 (CacheSize).
    int waiting = 0;
    for (const auto& w : waiting_) waiting += static_cast<int>(w->size());
    const int inflight = inflight_.load();
    metrics_->set_gauge("scheduler_scheduler_goroutines", "work=\"binding\"",
                        static_cast<double>(std::max(0, inflight - waiting)));
    metrics_->set_gauge("scheduler_scheduler_goroutines", "work=\"permit\"", static_cast<double>(waiting));
    metrics_->set_gauge("scheduler_scheduler_cache_size", "type=\"assumed_pods\"", static_cast<double>(cache_->assumed_count()));
    metrics_->set_gauge("scheduler_scheduler_cache_size", "type=\"pods\"", static_cast<double>(cache_->pod_count()));
    metrics_->set_gauge("scheduler_scheduler_cache_size", "type=\"nodes\"", static_cast<double>(cache_->node_count()));
  }));
  informer_thread_ = std::thread([this] {
    name_this_thread("xs-informer");
    informer_loop();
  });
  sched_thread_ = std::thread([this] {
    name_this_thread("xs-sched");
    scheduling_loop();
  });
}

void Scheduler::stop() {
  bool was_running = running_.exchange(false);
  if (watcher_) {
    store_->unwatch(watcher_);
  }
  queue_->close();
  if (informer_thread_.joinable()) informer_thread_.join();
  if (sched_thread_.joinable()) sched_thread_.join();
  for (uint64_t id : timer_ids_) timers_->cancel(id);
  timer_ids_.clear();
  for (auto& w : waiting_) w->reject_all("scheduler stopped");
  if (binder_) binder_->stop();
  if (status_writer_) status_writer_->stop();
  if (was_running)
    for (auto& fw : frameworks_) fw->stop();
  timers_->stop();
}

Framework* Scheduler::framework_for(const std::string& scheduler_name) {
  auto it = by_name_.find(scheduler_name);
  return it == by_name_.end() ? nullptr : it->second;
}

bool Scheduler::responsible_for(const Pod& p) const { return by_name_.count(p.scheduler_name) > 0; }

Scheduler::Stats Scheduler::stats() const {
  Stats st;
  auto rd = [](const std::atomic<uint64_t>& a) { return a.load(std::memory_order_relaxed); };
  st.attempts = rd(cnt_.attempts);
  st.scheduled = rd(cnt_.scheduled);
  st.unschedulable = rd(cnt_.unschedulable);
  st.errors = rd(cnt_.errors);
  st.bound = rd(cnt_.bound);
  st.bind_failures = rd(cnt_.bind_failures);
  st.preemption_attempts = rd(cnt_.preemption_attempts);
  st.eq_filter_hits = rd(cnt_.eq_filter_hits);
  st.eq_filter_misses = rd(cnt_.eq_filter_misses);
  st.scan_memo_served = rd(cnt_.scan_memo_served);
  st.scan_memo_mismatches = rd(cnt_.scan_memo_mismatches);
  return st;
}

std::vector<GangRecord> Scheduler::gang_records(bool clear) {
  std::lock_guard<std::mutex> g(stats_mu_);
  std::vector<GangRecord> out(gang_done_.begin(), gang_done_.end());
  if (clear) gang_done_.clear();
  return out;
}

// ------------------------------------------------------------- informers ----
void Scheduler::informer_loop() {
  while (running_.load()) {
    auto evs = watcher_->next(50, 8192);
    if (evs.empty()) continue;
    int64_t batch_start = tracer_.enabled() ? clock_->now_us() : 0;
    // The batch is handled in windows of >= informer_window_ events that end
    // on a PodGroup boundary, so the scheduling thread starts on the first
    // gangs of a bulk create instead of waiting for the whole batch.
    // Per window, pass 1 parses every pod once and publishes it to the
    // listers, so a PreFilter racing the window sees every sibling of a
    // PodGroup created together (Coscheduling counts them); pass 2 then
    // drives cache and queue.
    std::vector<PodPtr> parsed(evs.size());
    std::vector<PodPtr> prev(evs.size());
    std::vector<size_t> to_parse;
    auto group_of = [](const WatchEvent& ev) -> const std::string& {
      return (*ev.obj)["metadata"]["labels"][kPodGroupLabel].as_string();
    };
    size_t lo = 0;
    while (lo < evs.size()) {
      size_t hi = lo;
      while (hi < evs.size()) {
        const auto& ev = evs[hi];
        if (hi - lo >= informer_window_) {
          const auto& pe = evs[hi - 1];
          bool same_group = ev.kind == "pods" && pe.kind == "pods" && ev.type == EventType::Added &&
                            pe.type == EventType::Added && !group_of(ev).empty() && group_of(ev) == group_of(pe);
          if (!same_group) break;
        }
        ++hi;
        if (ev.kind != "pods" || ev.type == EventType::Deleted) continue;
        try {
          if (ev.type == EventType::Modified) parsed[hi - 1] = copy_for_modified(ev);
        } catch (const std::exception&) {
          continue;
        }
        if (!parsed[hi - 1]) to_parse.push_back(hi - 1);
      }
      // Pod::from_json is pure: a window's parses run on the parse helpers.
      if (!to_parse.empty()) {
        auto parse_one = [&](int k) {
          const size_t i = to_parse[static_cast<size_t>(k)];
          try {
            parsed[i] = Pod::from_json(*evs[i].obj, *gpu_names_);
          } catch (const std::exception&) {
            // left unparsed: handle_event below parses it again and reports
          }
        };
        if (parse_pool_) {
          parse_pool_->until(static_cast<int>(to_parse.size()), parse_one, nullptr, &parse_site_);
        } else {
          for (size_t k = 0; k < to_parse.size(); ++k) parse_one(static_cast<int>(k));
        }
        to_parse.clear();
      }
      // The window's pods enter the listers under one lock (previous objects back).
      informers_->upsert_pods(&parsed[lo], &prev[lo], hi - lo);
      for (size_t i = lo; i < hi;) {
        if (!parsed[i] && evs[i].type == EventType::Deleted && evs[i].kind == "pods") {
          size_t j = i + 1;
          while (j < hi && evs[j].type == EventType::Deleted && evs[j].kind == "pods") ++j;
          if (j - i > 1) {
            handle_pod_deletes(&evs[i], j - i);
            i = j;
            continue;
          }
        }
        if (parsed[i])
          handle_parsed_pod_event(evs[i], parsed[i], prev[i]);
        else
          handle_event(evs[i]);
        parsed[i].reset();
        prev[i].reset();
        ++i;
      }
      lo = hi;
    }
    if (tracer_.enabled() && batch_start)
      tracer_.record(TraceEvent{"informer_batch", std::to_string(evs.size()) + " events", "", batch_start,
                                clock_->now_us() - batch_start, 2});
  }
}

size_t Scheduler::sync_informers(int timeout_ms) {
  size_t n = 0;
  for (;;) {
    auto evs = watcher_->next(n == 0 ? timeout_ms : 0, 8192);
    if (evs.empty()) break;
    for (const auto& ev : evs) handle_event(ev);
    n += evs.size();
  }
  return n;
}

void Scheduler::handle_event(const WatchEvent& ev) {
  try {
    if (ev.kind == "pods") {
      handle_pod_event(ev);
    } else if (ev.kind == "nodes") {
      handle_node_event(ev);
    } else {
      const Json& o = *ev.obj;
      bool del = ev.type == EventType::Deleted;
      if (ev.kind == "podgroups") {
        if (del) {
          // A deletion needs the key only (no parse: a wave tears down
          // hundreds of groups at once).
          const Json& md = o["metadata"];
          const std::string key = md["namespace"].as_string() + "/" + md["name"].as_string();
          informers_->delete_pod_group(key);
          // A gang deleted before it was admitted leaves no open record: a
          // later PodGroup of the same name starts its own timeline.
          std::lock_guard<std::mutex> g(stats_mu_);
          gangs_.erase(key);
        } else {
          informers_->upsert_pod_group(PodGroup::from_json(o));
        }
      } else if (ev.kind == "elasticquotas") {
        auto eq = ElasticQuota::from_json(o);
        if (del) informers_->delete_elastic_quota(eq->meta.key()); else informers_->upsert_elastic_quota(eq);
      } else if (ev.kind == "noderesourcetopologies") {
        auto n = NodeResourceTopology::from_json(o);
        if (del) informers_->delete_nrt(n->meta.name); else informers_->upsert_nrt(n);
        cache_->set_nrt(n->meta.name, del ? nullptr : n);
      } else if (ev.kind == "poddisruptionbudgets") {
        auto p = PodDisruptionBudget::from_json(o);
        if (del) informers_->delete_pdb(p->meta.key()); else informers_->upsert_pdb(p);
      } else if (ev.kind == "priorityclasses") {
        auto pc = PriorityClass::from_json(o);
        if (del) informers_->delete_priority_class(pc->meta.name); else informers_->upsert_priority_class(pc);
      } else if (ev.kind == "persistentvolumes") {
        auto pv = PersistentVolume::from_json(o);
        if (del) informers_->delete_pv(pv->meta.name); else informers_->upsert_pv(pv);
      } else if (ev.kind == "persistentvolumeclaims") {
        auto pvc = PersistentVolumeClaim::from_json(o);
        if (del) informers_->delete_pvc(pvc->meta.key()); else informers_->upsert_pvc(pvc);
      } else if (ev.kind == "storageclasses") {
        auto sc = StorageClass::from_json(o);
        if (del) informers_->delete_storage_class(sc->meta.name); else informers_->upsert_storage_class(sc);
      } else if (ev.kind == "csinodes") {
        auto n = CSINode::from_json(o);
        if (del) informers_->delete_csinode(n->meta.name); else informers_->upsert_csinode(n);
      }
      for (auto& fw : frameworks_) fw->dispatch_object_event(ev.kind, static_cast<int>(ev.type), ev.obj, ev.old);
      queue_->move_all_to_active_or_backoff(ClusterEvent{resource_for_kind(ev.kind), action_for(ev.type), ""});
    }
  } catch (const std::exception& e) {
    // A malformed object must not kill the informer thread.
    report_informer_error(ev, e.what());
  }
}

// The object is dropped from the scheduler's view: say so (log line and, for
// pods and nodes, a Warning event on the object) so that, e.g., a pod naming
// a 65th distinct resource does not just silently stay Pending.
void Scheduler::report_informer_error(const WatchEvent& ev, const char* what) {
  metrics_->inc("xsched_informer_errors_total", "kind=\"" + ev.kind + "\"");
  std::string ns, name;
  if (ev.obj) {
    const Json& md = (*ev.obj)["metadata"];
    ns = md["namespace"].str_or("");
    name = md["name"].str_or("");
  }
  XS_WARN("informer dropped object").kv("kind", ev.kind).kv("namespace", ns).kv("name", name).kv("err", what);
  if (name.empty() || ev.type == EventType::Deleted) return;
  if (ev.kind == "pods" || ev.kind == "nodes") {
    try {
      client_->record_event(ev.kind == "pods" ? "Pod" : "Node", ns, name, "Warning", "FailedToDecode",
                            std::string("scheduler cannot use this object: ") + what);
    } catch (const std::exception&) {
    }
  }
}

// The pod a Deleted event removes. The lister copy stands in for the final
// state when it is the same pod on the same node (all deletion needs), saving
// a parse per delete.
PodPtr Scheduler::deleted_pod(const WatchEvent& ev) {
  const Json& md = (*ev.obj)["metadata"];
  PodPtr p = informers_->pod(md["namespace"].as_string(), md["name"].as_string());
  if (!p || p->uid() != md["uid"].as_string() || p->node_name != (*ev.obj)["spec"]["nodeName"].as_string())
    p = Pod::from_json(*ev.obj, *gpu_names_);
  return p;
}

void Scheduler::forget_unassigned_pod(const Pod& p) {
  queue_->remove(p);
  for (auto& w : waiting_)
    if (auto wp = w->get(p.uid())) wp->reject("", "pod " + p.key() + " was deleted");
  // An assumed-but-unbound pod may still sit in the cache.
  if (cache_->is_assumed(p.uid())) {
    if (auto cached = cache_->get_pod(p.uid())) {
      cache_->forget_pod(*cached);
      queue_->move_all_to_active_or_backoff(ClusterEvent{"Pod", kDelete, "AssignedPodDelete"});
      capacity_freed();
    }
  }
}

void Scheduler::capacity_freed() {
  for (auto& fw : frameworks_) fw->notify_capacity_freed();
}

void Scheduler::handle_pod_deletes(const WatchEvent* evs, size_t n) {
  std::vector<PodPtr> gone, assigned;
  gone.reserve(n);
  assigned.reserve(n);
  // One lister lock for the run: keys out, lister objects back where they
  // still describe the deleted pod (no parse for those).
  std::vector<std::string> keys;
  std::vector<std::string_view> uids, nodes;
  std::vector<size_t> idx;
  keys.reserve(n);
  uids.reserve(n);
  nodes.reserve(n);
  idx.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    try {
      for (auto& fw : frameworks_) fw->dispatch_object_event("pods", static_cast<int>(evs[i].type), evs[i].obj, evs[i].old);
      const Json& o = *evs[i].obj;
      const Json& md = o["metadata"];
      const std::string& ns = md["namespace"].as_string();
      const std::string& name = md["name"].as_string();
      std::string key;
      key.reserve(ns.size() + 1 + name.size());
      key.append(ns).push_back('/');
      key.append(name);
      keys.push_back(std::move(key));
      uids.push_back(md["uid"].as_string());
      nodes.push_back(o["spec"]["nodeName"].as_string());
      idx.push_back(i);
    } catch (const std::exception& e) {
      report_informer_error(evs[i], e.what());
    }
  }
  std::vector<PodPtr> listed = informers_->take_pods(keys, uids, nodes);
  for (size_t k = 0; k < idx.size(); ++k) {
    try {
      PodPtr p = listed[k] ? std::move(listed[k]) : Pod::from_json(*evs[idx[k]].obj, *gpu_names_);
      if (!p->node_name.empty()) assigned.push_back(p);
      gone.push_back(std::move(p));
    } catch (const std::exception& e) {
      report_informer_error(evs[idx[k]], e.what());
    }
  }
  if (!assigned.empty()) {
    cache_->remove_pods(assigned);
    queue_->move_all_to_active_or_backoff(ClusterEvent{"Pod", kDelete, "AssignedPodDelete"});
    capacity_freed();
  }
  for (const auto& p : gone)
    if (p->node_name.empty()) forget_unassigned_pod(*p);
  // The lister's and the cache's references are gone: the last ones to the
  // wave's Pod objects are here, freed off the informer thread.
  assigned.clear();
  defer_destroy(std::make_shared<std::vector<PodPtr>>(std::move(gone)));
}

void Scheduler::handle_pod_event(const WatchEvent& ev) {
  for (auto& fw : frameworks_) fw->dispatch_object_event("pods", static_cast<int>(ev.type), ev.obj, ev.old);
  if (ev.type == EventType::Deleted) {
    PodPtr p = deleted_pod(ev);
    informers_->delete_pod(*p);
    if (!p->node_name.empty()) {
      cache_->remove_pod(*p);
      queue_->move_all_to_active_or_backoff(ClusterEvent{"Pod", kDelete, "AssignedPodDelete"});
      capacity_freed();
    } else {
      forget_unassigned_pod(*p);
    }
    return;
  }
  PodPtr np = ev.type == EventType::Modified ? copy_for_modified(ev) : nullptr;
  if (!np) np = Pod::from_json(*ev.obj, *gpu_names_);
  PodPtr old = informers_->pod(np->ns(), np->name());
  informers_->upsert_pod(np);
  apply_pod_update(ev, np, old);
}

// The Modified event of our own Binding: the new object is the version the
// pod was assumed from plus nodeName, the Reserve annotations, the
// PodScheduled condition and a resourceVersion. When the previous version is
// exactly the one the assumed copy came from (same resourceVersion), the
// informer's object is built by copying the assumed pod and refreshing those
// fields, instead of parsing the whole Pod again (one parse per pod, not two).
PodPtr Scheduler::bound_copy_of_assumed(const WatchEvent& ev) {
  if (!ev.old) return nullptr;
  const Json& obj = *ev.obj;
  const Json& spec = obj["spec"];
  const std::string& node = spec["nodeName"].as_string();
  if (node.empty() || !(*ev.old)["spec"]["nodeName"].as_string().empty()) return nullptr;
  const Json& md = obj["metadata"];
  PodPtr assumed = cache_->get_pod(md["uid"].as_string());
  if (!assumed || !cache_->is_assumed(assumed->uid()) || assumed->node_name != node) return nullptr;
  const Json& old_rv = (*ev.old)["metadata"]["resourceVersion"];
  int64_t from_rv = old_rv.is_string() ? std::atoll(old_rv.as_string().c_str()) : old_rv.as_int();
  if (from_rv != assumed->meta.resource_version) return nullptr;  // updated since the cycle: parse
  if (md["annotations"].size() != assumed->meta.annotations.size()) return nullptr;
  auto np = std::make_shared<Pod>(*assumed);
  const Json& rv = md["resourceVersion"];
  np->meta.resource_version = rv.is_string() ? std::atoll(rv.as_string().c_str()) : rv.as_int();
  np->template_hash = 0;  // as Pod::from_json for an assigned pod
  const Json& status = obj["status"];
  np->phase = status["phase"].is_string() ? status["phase"].as_string() : std::string("Pending");
  np->nominated_node_name = status["nominatedNodeName"].as_string();
  np->start_time = status["startTime"].is_string() ? parse_rfc3339(status["startTime"].as_string()) : 0;
  np->scheduled_at = 0;
  for (const auto& c : status["conditions"].items())
    if (c["type"].as_string() == "PodScheduled" && c["status"].as_string() == "True")
      np->scheduled_at = parse_rfc3339(c["lastTransitionTime"].as_string());
  return np;
}

// A failed cycle's PodScheduled=False patch (handle_failure) changes status
// only; at saturation thousands of them reach the informer while creations and
// deletions queue behind them. The lister's object for the previous version
// is copied and its status fields refreshed (the fields Pod::from_json reads
// from status) instead of parsing the pod again.
PodPtr Scheduler::status_copy_of_listed(const WatchEvent& ev) {
  if (!ev.status_only || !ev.old) return nullptr;
  const Json& obj = *ev.obj;
  const Json& md = obj["metadata"];
  PodPtr listed = informers_->pod(md["namespace"].as_string(), md["name"].as_string());
  if (!listed || listed->uid() != md["uid"].as_string()) return nullptr;
  const Json& old_rv = (*ev.old)["metadata"]["resourceVersion"];
  const int64_t from_rv = old_rv.is_string() ? std::atoll(old_rv.as_string().c_str()) : old_rv.as_int();
  if (from_rv != listed->meta.resource_version) return nullptr;  // the lister holds another version: parse
  auto np = std::make_shared<Pod>(*listed);
  const Json& rv = md["resourceVersion"];
  np->meta.resource_version = rv.is_string() ? std::atoll(rv.as_string().c_str()) : rv.as_int();
  const Json& status = obj["status"];
  np->phase = status["phase"].is_string() ? status["phase"].as_string() : std::string("Pending");
  np->nominated_node_name = status["nominatedNodeName"].as_string();
  np->start_time = status["startTime"].is_string() ? parse_rfc3339(status["startTime"].as_string()) : 0;
  np->scheduled_at = 0;
  for (const auto& c : status["conditions"].items())
    if (c["type"].as_string() == "PodScheduled" && c["status"].as_string() == "True")
      np->scheduled_at = parse_rfc3339(c["lastTransitionTime"].as_string());
  return np;
}

void Scheduler::handle_parsed_pod_event(const WatchEvent& ev, const PodPtr& np, PodPtr old) {
  try {
    for (auto& fw : frameworks_) fw->dispatch_object_event("pods", static_cast<int>(ev.type), ev.obj, ev.old);
    apply_pod_update(ev, np, std::move(old));
  } catch (const std::exception& e) {
    report_informer_error(ev, e.what());
  }
}

void Scheduler::apply_pod_update(const WatchEvent& ev, const PodPtr& np, PodPtr old) {
  if (old && old->uid() != np->uid()) old = nullptr;  // recreated with same name
  bool assigned = !np->node_name.empty();
  if (ev.type == EventType::Added || !old) {
    if (assigned) {
      cache_->add_pod(np);
      queue_->assigned_pod_added(*np);
    } else if (responsible_for(*np) && !np->terminating()) {
      // The gang record first: once queued, the pod can be scheduled, admitted
      // and bound by other threads before this one runs again, and a record
      // opened after its own completion would never close (the gang would
      // read as never bound).
      note_gang_enqueue(*np, clock_->now_us());
      queue_->add(np);
      // A new member may complete its PodGroup: re-activate siblings parked
      // in unschedulableQ/backoffQ (targeted form of the Pod/Add cluster
      // event Coscheduling registers; O(group size), not O(queue)).
      if (!np->pod_group.empty()) {
        std::vector<PodPtr> sib = informers_->pods_in_group_of(*np);
        sib.erase(std::remove_if(sib.begin(), sib.end(),
                                 [&](const PodPtr& q) { return q->uid() == np->uid() || !q->node_name.empty(); }),
                  sib.end());
        if (!sib.empty()) queue_->activate(sib);
      }
    }
    return;
  }
  bool was_assigned = !old->node_name.empty();
  if (was_assigned && assigned) {
    cache_->update_pod(old, np);
    queue_->assigned_pod_updated(*np);
  } else if (!was_assigned && assigned) {
    queue_->remove(*old);
    cache_->add_pod(np);
    queue_->assigned_pod_added(*np);
  } else if (!assigned && responsible_for(*np)) {
    if (np->terminating()) {
      queue_->remove(*np);
    } else if (!cache_->is_assumed(np->uid())) {
      queue_->update(old, np);
    }
  }
}

void Scheduler::handle_node_event(const WatchEvent& ev) {
  for (auto& fw : frameworks_) fw->dispatch_object_event("nodes", static_cast<int>(ev.type), ev.obj, ev.old);
  if (ev.type == EventType::Deleted) {
    auto n = Node::from_json(*ev.obj, *gpu_names_);
    cache_->remove_node(n->name());
    return;
  }
  auto n = Node::from_json(*ev.obj, *gpu_names_);
  if (ev.type == EventType::Added || !ev.old) {
    cache_->add_node(n);
    queue_->move_all_to_active_or_backoff(ClusterEvent{"Node", kAdd, "NodeAdd"});
    capacity_freed();
    return;
  }
  auto o = Node::from_json(*ev.old, *gpu_names_);
  cache_->update_node(n);
  uint32_t action = 0;
  if (!(o->allocatable == n->allocatable)) action |= kUpdateNodeAllocatable;
  if (o->meta.labels != n->meta.labels) action |= kUpdateNodeLabel;
  if (o->taints.size() != n->taints.size() || o->unschedulable != n->unschedulable) action |= kUpdateNodeTaint;
  else
    for (size_t i = 0; i < o->taints.size(); ++i)
      if (o->taints[i].key != n->taints[i].key || o->taints[i].value != n->taints[i].value ||
          o->taints[i].effect != n->taints[i].effect)
        action |= kUpdateNodeTaint;
  if (o->meta.annotations != n->meta.annotations) action |= kUpdateNodeLabel;  // GPU topology annotation
  if (action) queue_->move_all_to_active_or_backoff(ClusterEvent{"Node", action, "NodeUpdate"});
  if (action & kUpdateNodeAllocatable) capacity_freed();
}

// -------------------------------------------------------- gang tracking ----
namespace {
// "ns/group" in a per-thread buffer: gang bookkeeping runs per pod and a
// lookup must not allocate a key string.
const std::string& gang_key(const Pod& p) {
  thread_local std::string k;
  k.assign(p.ns());
  k.push_back('/');
  k.append(p.pod_group);
  return k;
}
}  // namespace

void Scheduler::note_gang_enqueue(const Pod& p, int64_t t) {
  if (p.pod_group.empty()) return;
  const std::string& key = gang_key(p);
  std::lock_guard<std::mutex> g(stats_mu_);
  auto it = gangs_.find(key);
  if (it != gangs_.end()) return;
  GangRecord& r = gangs_[key];
  r.pg = key;
  r.first_enqueue_us = t;
}

void Scheduler::note_gang_event(const Pod& p, bool bound) {
  if (p.pod_group.empty()) return;
  auto pg = informers_->pod_group_of(p);
  if (!pg) return;
  int need = std::max(1, pg->min_member);
  const std::string& key = gang_key(p);
  std::lock_guard<std::mutex> g(stats_mu_);
  auto it = gangs_.find(key);
  if (it == gangs_.end()) return;
  GangRecord& r = it->second;
  r.size = need;
  int64_t now = clock_->now_us();
  if (!bound) {
    if (r.admit_us == 0) r.admit_us = now;
    return;
  }
  const uint64_t nh = std::hash<std::string_view>{}(std::string_view(p.node_name));
  if (std::find(r.nodes.begin(), r.nodes.end(), nh) == r.nodes.end()) r.nodes.push_back(nh);
  if (++r.bound < need) return;
  r.bound_us = now;
  if (r.admit_us == 0) r.admit_us = now;
  // The per-size histogram, looked up once per size and metrics epoch.
  const uint64_t epoch = metrics_->epoch();
  if (gang_hist_epoch_ != epoch) {
    gang_hist_.clear();
    gang_hist_epoch_ = epoch;
  }
  Histogram*& hist = gang_hist_[need];
  if (!hist) hist = &metrics_->histogram("xsched_gang_admit_seconds", "size=\"" + std::to_string(need) + "\"");
  hist->observe(static_cast<double>(r.bound_us - r.first_enqueue_us) / 1e6);
  gang_done_.push_back(r);
  gangs_.erase(it);
}

void Scheduler::note_gang_planned(const Pod& p, bool hostable) {
  if (p.pod_group.empty()) return;
  const std::string& key = gang_key(p);
  std::lock_guard<std::mutex> g(stats_mu_);
  auto it = gangs_.find(key);
  if (it != gangs_.end()) it->second.hostable = hostable ? 1 : 0;
}

// Why was a gang denied? The cache's view (free SPX GPUs, those held by
// assumed pods of gangs still waiting at Permit) against the store's at the
// same moment (bound pods only): separates a stale cache (deletions not yet
// observed) from GPUs held by other waiting gangs and from a real shortage.
void Scheduler::note_gang_denied(const Pod& p, const char* why) {
  {
    std::lock_guard<std::mutex> g(stats_mu_);
    ++gang_denials_total_;
    if (gang_denials_.size() >= kMaxGangDenials) return;
  }
  GangDenial d;
  d.pg = gang_key(p);
  d.why = why;
  d.t_us = clock_->now_us();
  auto pg = informers_->pod_group_of(p);
  d.min_member = pg ? pg->min_member : 0;
  d.assigned = cache_->assigned_in_group(p.pg_key);
  for (const auto& w : waiting_) d.waiting_at_permit += static_cast<int>(w->size());
  d.in_binding = std::max(0, inflight_.load() - d.waiting_at_permit);
  d.need_gpus = p.gpu_demand.kind == GpuDemand::Gpu ? p.gpu_demand.amount : 0;
  std::unordered_map<std::string, int> spx;
  for (const auto& r : cache_->gpu_census()) {
    spx[r.node] = r.spx;
    d.cache_free += r.free_whole;
    d.cache_max_node_free = std::max(d.cache_max_node_free, r.free_whole);
    d.assumed_held += r.assumed_whole;
  }
  if (store_ && opts_.gang_denial_census) {
    std::unordered_map<std::string, int> used;
    const std::string& gpu = gpu_names_->gpu;
    for (const auto& po : store_->list("pods", "")) {
      const Json& spec = (*po)["spec"];
      const std::string& node = spec["nodeName"].as_string();
      if (node.empty() || (*po)["metadata"].get("deletionTimestamp")) continue;
      int64_t n = 0;
      for (const auto& c : spec["containers"].items()) {
        const Json& lim = c["resources"]["limits"][gpu];
        if (lim.is_string()) n += Quantity::parse(lim.as_string()).value();
        else if (lim.is_number()) n += lim.as_int();
      }
      if (n) used[node] += static_cast<int>(n);
    }
    d.store_free = 0;
    for (const auto& [node, cap] : spx) {
      auto u = used.find(node);
      int f = std::max(0, cap - (u == used.end() ? 0 : u->second));
      d.store_free += f;
      d.store_max_node_free = std::max(d.store_max_node_free, f);
    }
  }
  // The gang still needed (min_member - assigned) more whole GPUs. GPUs free
  // in the store are either truly taken by pods in flight (waiting at Permit
  // or being bound: not yet bound in the store) or seen as used only by a
  // cache that has not observed the deletions yet.
  // Without the store census the cache alone separates GPUs held by pods in
  // flight (assumed, not yet bound) from a shortage of bound pods.
  const int64_t missing = d.need_gpus * std::max(0, d.min_member - d.assigned);
  const int64_t in_flight = d.need_gpus * (d.waiting_at_permit + d.in_binding);  // GPUs, not pods
  if (d.need_gpus == 0) d.cause = "not_whole_gpu";
  else if (d.store_free < 0)
    d.cause = d.cache_free >= missing ? "placement"
              : d.cache_free + d.assumed_held >= missing ? "held_by_gangs_in_flight"
                                                         : "capacity";
  else if (d.store_free < missing) d.cause = "capacity";
  else if (d.store_free - in_flight < missing) d.cause = "held_by_gangs_in_flight";
  else if (d.cache_free < missing) d.cause = "stale_cache";
  else d.cause = "placement";
  std::lock_guard<std::mutex> g(stats_mu_);
  if (gang_denials_.size() < kMaxGangDenials) gang_denials_.push_back(std::move(d));
}

uint64_t Scheduler::gang_parks(bool clear) {
  return clear ? gang_parks_total_.exchange(0) : gang_parks_total_.load();
}

std::vector<GangDenial> Scheduler::gang_denials(bool clear, uint64_t* total) {
  std::lock_guard<std::mutex> g(stats_mu_);
  std::vector<GangDenial> out = gang_denials_;
  if (total) *total = gang_denials_total_;
  if (clear) {
    gang_denials_.clear();
    gang_denials_total_ = 0;
  }
  return out;
}

// -------------------------------------------------------- scheduling ----
double Scheduler::loop_age_seconds() const {
  int64_t t = loop_tick_us_.load(std::memory_order_relaxed);
  if (!t || !running_.load()) return 0.0;
  return static_cast<double>(RealClock().now_us() - t) / 1e6;
}

void Scheduler::scheduling_loop() {
  RealClock rc;
  while (running_.load()) {
    loop_tick_us_.store(rc.now_us(), std::memory_order_relaxed);
    auto qpi = queue_->pop(100);
    if (!qpi) continue;
    std::lock_guard<std::mutex> g(sched_mu_);
    in_cycle_.fetch_add(1);
    schedule_cycle(qpi);
    in_cycle_.fetch_sub(1);
  }
}

bool Scheduler::schedule_one(int timeout_ms) {
  auto qpi = queue_->pop(timeout_ms);
  if (!qpi) return false;
  std::lock_guard<std::mutex> g(sched_mu_);
  in_cycle_.fetch_add(1);
  schedule_cycle(qpi);
  in_cycle_.fetch_sub(1);
  return true;
}

bool Scheduler::wait_idle(int timeout_ms) {
  int64_t deadline = clock_->now_us() + static_cast<int64_t>(timeout_ms) * 1000;
  RealClock rc;
  int64_t real_deadline = rc.now_us() + static_cast<int64_t>(timeout_ms) * 1000;
  for (;;) {
    auto c = queue_->counts();
    size_t waiting = 0;
    for (auto& w : waiting_) waiting += w->size();
    // Idle includes the FailedScheduling event writer: after an overload its
    // backlog would otherwise keep writing into the next measurement.
    if (c.active == 0 && c.backoff == 0 && waiting == 0 && inflight_.load() == 0 && in_cycle_.load() == 0 &&
        watcher_->pending() == 0 && (!status_writer_ || status_writer_->pending() == 0))
      return true;
    if (rc.now_us() > real_deadline && clock_->now_us() > deadline) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

int Scheduler::num_feasible_nodes_to_find(Framework& fw, int n) const {
  constexpr int kMinFeasible = 100;       // generic_scheduler.go:47
  constexpr int kMinPercentage = 5;
  int pct = fw.config().percentage_of_nodes_to_score;
  if (n < kMinFeasible || pct >= 100) return n;
  int adaptive = pct;
  if (adaptive <= 0) {
    adaptive = 50 - n / 125;
    if (adaptive < kMinPercentage) adaptive = kMinPercentage;
  }
  int num = n * adaptive / 100;
  if (num < kMinFeasible) return kMinFeasible;
  return num;
}

// Replaced snapshot versions may hold the last reference to deleted pods;
// free them in batches on a binder thread instead of in the scheduling cycle.
void Scheduler::run_bind_task(BindTask* t) {
  std::shared_ptr<BindTask> hold = std::move(t->keep);
  t->self->binding_cycle(*t, t->permit_status);
}

void Scheduler::release_retired() {
  if (snapshot_.retired.size() >= 32) {
    // The batch is released on a binder thread; its emptied vector comes back
    // through retired_spare_ with its capacity (no allocation per batch).
    auto batch = std::make_shared<std::vector<NodeInfoPtr>>(std::move(snapshot_.retired));
    snapshot_.retired.clear();
    {
      std::lock_guard<std::mutex> g(retired_spare_mu_);
      if (!retired_spare_.empty()) {
        snapshot_.retired.swap(retired_spare_.back());
        retired_spare_.pop_back();
      }
    }
    if (snapshot_.retired.capacity() < 64) snapshot_.retired.reserve(64);
    binder_->submit([this, batch] {
      batch->clear();
      std::lock_guard<std::mutex> g(retired_spare_mu_);
      if (retired_spare_.size() < 8) retired_spare_.push_back(std::move(*batch));
    });
  }
  if (snapshot_.retired_deltas.size() >= 256) {
    auto batch = std::make_shared<std::vector<PodDelta>>(std::move(snapshot_.retired_deltas));
    snapshot_.retired_deltas.clear();
    snapshot_.retired_deltas.reserve(512);
    binder_->submit([batch] { batch->clear(); });
  }
}

// Which snapshot positions carry nominated pods: rebuilt from the view when
// the view object or the node set changed, else updated for the nodes the
// view's change log touched (a preemption wave keeps hundreds of pods
// nominated; re-deriving every position per cycle was a hash lookup each).
// Stale marks only send a node down the exact (uncached) path; every node
// nominated in the view is always marked.
void Scheduler::refresh_nom_mark(const NominatedMap* view) {
  if (!view || view->empty()) {
    nom_mark_valid_ = false;
    return;
  }
  const size_t n = snapshot_.nodes.size();
  auto mark = [&](const std::string& node) {
    auto it = snapshot_.index.find(node);
    if (it == snapshot_.index.end()) return;
    auto vit = view->find(node);
    const bool on = vit != view->end() && !vit->second.empty();
    nom_mark_[it->second] = on;
    nom_list_[it->second] = on ? &vit->second : nullptr;  // map nodes do not move
  };
  if (!nom_mark_valid_ || view != nom_src_ || snapshot_.node_epoch != nom_epoch_ || nom_mark_.size() != n) {
    nom_mark_.assign(n, 0);
    nom_list_.assign(n, nullptr);
    for (const auto& [node, pods] : *view)
      if (!pods.empty()) mark(node);
  } else {
    for (const auto& node : nom_changed_) mark(node);
  }
  nom_changed_.clear();
  nom_src_ = view;
  nom_epoch_ = snapshot_.node_epoch;
  nom_mark_valid_ = true;
}

Scheduler::EqEntry* Scheduler::eq_entry(Framework& fw, const Pod& p) {
  if (!opts_.equivalence_cache || p.template_hash == 0) return nullptr;
  auto& per_fw = eq_[&fw];
  auto& e = per_fw[p.template_hash];
  if (!e) {
    if (per_fw.size() > 256) {  // bounded: drop every template (they refill on demand)
      per_fw.clear();
      return eq_entry(fw, p);
    }
    e = std::make_unique<EqEntry>();
  }
  if (e->epoch != snapshot_.node_epoch || e->table.n != snapshot_.nodes.size()) {
    e->epoch = snapshot_.node_epoch;
    e->table.reset(snapshot_.nodes.size());
    e->scan.valid = false;
  }
  return e.get();
}

namespace {

// "0/N nodes are available: k reason, ..." over a complete diagnosis.
std::string fit_error_message(int n, const NodeStatusMap& m) {
  std::map<std::string, int> reasons;
  m.for_each([&](std::string_view, const Status& st) {
    for (const auto& r : st.reasons()) ++reasons[r];
  });
  std::string msg = "0/" + std::to_string(n) + " nodes are available:";
  bool first = true;
  for (const auto& kv : reasons) {
    msg += (first ? " " : ", ") + std::to_string(kv.second) + " " + kv.first;
    first = false;
  }
  return msg + ".";
}

}  // namespace

Status Scheduler::find_nodes_that_fit(Framework& fw, CycleState& s, const Pod& p, Diagnosis& d, NodeList& feasible,
                                      EqEntry* eq, bool full_diagnosis, std::vector<int>* feasible_pos) {
  // Extenders filter after the plugins; the diagnosis must then be complete,
  // since the FitError may come from nodes only an extender rejected.
  const bool ext = extenders_interested(p);
  full_diagnosis = full_diagnosis || ext;
  int64_t pf0 = tracer_.enabled() ? clock_->now_us() : 0;
  Status st = fw.run_pre_filter(s, p);
  if (tracer_.enabled()) tracer_.record(TraceEvent{"prefilter", p.key(), "", pf0, clock_->now_us() - pf0, 0});
  const auto& all = snapshot_.nodes;
  feasible.clear();
  if (feasible_pos) feasible_pos->clear();
  if (!st.is_success()) {
    if (!st.is_unschedulable()) return st;
    d.node_to_status.reserve(all.size());
    const bool fresh = d.node_to_status.empty();
    for (const auto& name : snapshot_.names) {
      if (fresh) d.node_to_status.append_unique(name, st);
      else d.node_to_status.emplace(name, st);
    }
    d.unschedulable_plugins.insert(st.failed_plugin());
    return Status(Code::Unschedulable, st.message()).with_plugin(st.failed_plugin());
  }
  // Prefer the nominated node (PreferNominatedNode, beta in 1.23).
  if (!p.nominated_node_name.empty()) {
    auto it = snapshot_.index.find(p.nominated_node_name);
    if (it != snapshot_.index.end()) {
      const NodeInfo* ni = all[it->second].get();
      Status nst = fw.run_filter_with_nominated_pods(s, p, *ni);
      if (nst.is_success()) {
        feasible.push_back(ni);
        if (feasible_pos) feasible_pos->push_back(static_cast<int>(it->second));
        if (!ext) return {};
        // evaluateNominatedNode: the extenders see the nominated node too;
        // when they reject it the full search below runs.
        Status es = run_extender_filters(p, feasible, feasible_pos, d);
        if (!es.is_success() || !feasible.empty()) return es;
      } else if (!nst.is_unschedulable()) {
        return nst;
      }
    }
  }
  int n = static_cast<int>(all.size());
  if (n == 0) return Status(Code::Unschedulable, "no nodes available to schedule pods");
  int to_find = num_feasible_nodes_to_find(fw, n);
  if (!fw.has(kFilter)) {
    for (int i = 0; i < std::min(n, to_find); ++i) {
      int pos = (next_start_node_ + i) % n;
      feasible.push_back(all[pos].get());
      if (feasible_pos) feasible_pos->push_back(pos);
    }
    next_start_node_ = (next_start_node_ + static_cast<int>(feasible.size())) % n;
    if (!ext) return {};
    Status es = run_extender_filters(p, feasible, feasible_pos, d);
    if (!es.is_success() || !feasible.empty()) return es;
    return Status(Code::Unschedulable, fit_error_message(n, d.node_to_status));
  }
  // A PreFilter node set (NodeRestriction, upstream's PreFilterResult; the
  // xGMI gang co-location plan of NodeResourceTopologyMatch): a short list is
  // evaluated directly, a larger set through a mask over the usual walk.
  const NodeRestriction* rs = s.read_as<NodeRestriction>(kNodeRestrictionKey);
  if (rs && rs->nodes != all.size()) rs = nullptr;  // planned for another node set
  if (rs && rs->list.empty() && rs->mask.empty()) {
    if (rs->fallback) {
      rs = nullptr;
    } else {  // nothing qualifies and the plugin allows no fallback
      d.node_to_status.reserve(all.size());
      const bool fresh = d.node_to_status.empty();
      for (const auto& name : snapshot_.names) {
        if (fresh) d.node_to_status.append_unique(name, rs->excluded);
        else d.node_to_status.emplace(name, rs->excluded);
      }
      d.unschedulable_plugins.insert(rs->excluded.failed_plugin());
      return Status(Code::Unschedulable, fit_error_message(n, d.node_to_status)).with_plugin(rs->excluded.failed_plugin());
    }
  }
  if (rs && rs->mask.empty()) {
    Status r = filter_listed(fw, s, p, d, feasible, eq, *rs, feasible_pos, ext);
    if (!r.is_success() && !r.is_unschedulable()) return r;
    if (!feasible.empty() || !rs->fallback) return r;
    d = Diagnosis{};  // none of the listed nodes fits: every node, as without the set
    feasible.clear();
    if (feasible_pos) feasible_pos->clear();
    rs = nullptr;
  }
  // The walk over the node window; `rmask` (may be null) excludes nodes
  // outside the PreFilter set (verdict rs->excluded, no Filter call).
  auto walk = [&](const char* rmask) -> Status {
    // Filter verdicts are reused only when every Filter plugin is node-local for
    // this pod. A node with nominated pods is evaluated with them added; that
    // verdict is cached too, keyed by the set of nominated pods that count for
    // this pod (Framework::nominated_signature), unless one of them reacts
    // with a PreFilter extension (the state would then not be node-local).
    bool eq_filter = eq && fw.filters_node_local(p, snapshot_);
    const char* nom_mark = nullptr;
    if (eq_filter && s.nominated && !s.nominated->empty()) {
      if (!nom_mark_valid_ || s.nominated.get() != nom_src_) refresh_nom_mark(s.nominated.get());
      nom_mark = nom_mark_.data();
    } else if (eq_filter && nominator_ && !nominator_->empty()) {
      // Nominations without this cycle's view (explain, or a caller that did
      // not snapshot them): no per-node knowledge, so no reuse.
      eq_filter = false;
    }
    int start = next_start_node_;
    // The members of one gang that share a pod template are evaluated over the
    // node window of the first of them (upstream rotates the window every
    // cycle, numFeasibleNodesToFind > 100 nodes): a rank then reuses its
    // sibling's Filter verdicts and node-local scores for every node but the
    // one the sibling took, and the gang's candidates are the same nodes
    // XGMIGangAffinity ranks.
    if (opts_.gang_window && !full_diagnosis && p.pg_key) {
      if (p.pg_key == window_gang_ && p.template_hash == window_tmpl_ && window_n_ == n) {
        start = window_start_;
      } else {
        window_gang_ = p.pg_key;
        window_tmpl_ = p.template_hash;
        window_start_ = start;
        window_n_ = n;
      }
    }
    // Per-node failures go to a position-indexed buffer (no lock, no map
    // insert per node); the NodeToStatusMap is only materialized when the
    // diagnosis is consumed: no feasible node (PostFilter / FitError) or explain.
    // Equivalence-cache verdicts are referenced in place, not copied: a Status
    // copy bumps the refcount of a failure status shared by every node, and 16
    // workers doing that per node serialize on its cache line.
    if (static_cast<int>(fail_buf_.size()) < n) fail_buf_.resize(n);
    fail_ptr_.assign(n, nullptr);
    Status first_err;
    bool has_err = false;
    int c = 0, processed = 0;
    uint64_t hits = 0;
    if (static_cast<int>(found_buf_.size()) < to_find + 1) found_buf_.resize(to_find + 1);
    if (static_cast<int>(found_pos_buf_.size()) < to_find + 1) found_pos_buf_.resize(to_find + 1);
    // One node's verdict: from the equivalence cache when it is valid for the
    // node's version (and, on a node with nominated pods, for the same set of
    // nominated pods), else computed into `own` or the cache slot.
    auto eval_node = [&](int pos, const NodeInfo& ni, Status& own, bool* hit) -> const Status* {
      if (rmask && !rmask[pos]) {
        *hit = true;
        return &rs->excluded;
      }
      if (!eq_filter) {
        own = fw.run_filter_with_nominated_pods(s, p, ni);
        return &own;
      }
      EqTable& t = eq->table;
      uint64_t sig = 0;
      bool cacheable = true;
      if (nom_mark && nom_mark[pos]) sig = fw.nominated_signature(s, p, nom_list_[pos], &cacheable);
      const int64_t gen = snapshot_.gen[pos];
      if (sig == 0) {  // no nominated pod counts for this pod: the plain verdict
        if (t.filter_gen[pos] == gen) {
          *hit = true;
        } else {
          t.filter[pos] = fw.run_filter(s, p, ni);
          t.filter_gen[pos] = gen;
        }
        return &t.filter[pos];
      }
      if (cacheable && t.nom_gen[pos] == gen && t.nom_sig[pos] == sig) {
        *hit = true;
        return &t.nom_filter[pos];
      }
      Status st = fw.run_filter_with_nominated_pods(s, p, ni);
      if (!cacheable) {
        own = std::move(st);
        return &own;
      }
      t.nom_filter[pos] = std::move(st);
      t.nom_gen[pos] = gen;
      t.nom_sig[pos] = sig;
      return &t.nom_filter[pos];
    };
    // The template's last scan of this window (EqEntry::scan): a gang rank
    // after its sibling re-evaluates only the scanned nodes whose version
    // changed since (usually the node the sibling took) and re-cuts the list at
    // numFeasibleNodesToFind, instead of walking the whole window again.
    EqEntry::ScanMemo* memo =
        (opts_.scan_memo && eq && eq_filter && !nom_mark && !full_diagnosis && !ext && !rmask) ? &eq->scan
                                                                                                  : nullptr;
    if (memo && !(memo->valid && memo->start == start && memo->n == n && memo->to_find == to_find &&
                  memo->epoch == snapshot_.node_epoch))
      memo->valid = false;
    const bool inline_ok = parallelizer_->plan_inline(n, &filter_site_);
    bool served = false;
    if (memo && memo->valid && inline_ok) {
      bool ok = true;
      int reevaluated = 0;
      const int m = memo->processed;
      auto at = [&](int off) { return start + off >= n ? start + off - n : start + off; };
      // The window is at most two contiguous runs of positions; each is checked
      // in blocks with memcmp, and only a block that differs element-wise.
      const int64_t* mg = memo->gens.data();
      const int64_t* sg = snapshot_.gen.data();
      constexpr int kBlock = 32;
      for (int off0 = 0; off0 < m && ok;) {
        const int pos0 = at(off0);
        const int run = std::min({m - off0, n - pos0, kBlock});
        if (std::memcmp(mg + off0, sg + pos0, static_cast<size_t>(run) * sizeof(int64_t)) != 0) {
          for (int j = 0; j < run && ok; ++j) {
            const int off = off0 + j, pos = pos0 + j;
            if (mg[off] == sg[pos]) continue;
            bool hit = false;
            const Status* fp = eval_node(pos, *all[pos], fail_buf_[pos], &hit);
            ++reevaluated;
            ok = fp->is_success() || fp->is_unschedulable();
            memo->ok[off] = fp->is_success();
            memo->gens[off] = sg[pos];
          }
        }
        off0 += run;
      }
      // Re-cut the list: branch-free appends (the buffers hold to_find + 1),
      // over the window's two contiguous runs ([start, n), then [0, ...)), with
      // every bound and base pointer in a local: a store to the int buffer
      // could alias `start`, whose address the lambdas above hold, and forced
      // a reload per node.
      int off = 0;
      if (ok) {
        const char* okv = memo->ok.data();
        const NodeInfoPtr* allp = all.data();
        const NodeInfo** fb = found_buf_.data();
        int* fpb = found_pos_buf_.data();
        const int s0 = start, nn = n, mm = m, want = to_find;
        int cc = c;
        for (int run = 0; run < 2 && off < mm && cc < want; ++run) {
          const int first_off = off;
          const int first_pos = run == 0 ? s0 : 0;
          const int end_off = run == 0 ? std::min(mm, nn - s0) : mm;
          for (; off < end_off && cc < want; ++off) {
            const int pos = first_pos + (off - first_off);
            fb[cc] = allp[pos].get();
            fpb[cc] = pos;
            cc += okv[off] != 0;
          }
        }
        c = cc;
      }
      for (; ok && c < to_find && off < n; ++off) {  // the scan has to reach further now
        const int pos = at(off);
        bool hit = false;
        const Status* fp = eval_node(pos, *all[pos], fail_buf_[pos], &hit);
        ++reevaluated;
        ok = fp->is_success() || fp->is_unschedulable();
        if (off < static_cast<int>(memo->gens.size())) {
          memo->gens[off] = snapshot_.gen[pos];
          memo->ok[off] = fp->is_success();
        } else {
          memo->gens.push_back(snapshot_.gen[pos]);
          memo->ok.push_back(fp->is_success());
        }
        if (fp->is_success()) {
          found_buf_[c] = all[pos].get();
          found_pos_buf_[c] = pos;
          ++c;
        }
      }
      if (ok && c > 0) {
        processed = off;
        memo->processed = off;
        hits = static_cast<uint64_t>(std::max(0, processed - reevaluated));
        served = true;
      } else {  // an error, or nothing feasible (the diagnosis needs every verdict): the full walk
        memo->valid = false;
        c = 0;
      }
    }
    if (served) {
      bool mismatch = false;
      if (opts_.scan_memo_verify) {  // the full walk must find the same nodes and stop at the same one
        int vc = 0, vp = 0;
        for (int i = 0; i < n && vc < to_find && !mismatch; ++i) {
          const int pos = start + i >= n ? start + i - n : start + i;
          bool hit = false;
          const Status* fp = eval_node(pos, *all[pos], fail_buf_[pos], &hit);
          ++vp;
          if (fp->is_success()) mismatch = vc >= c || found_pos_buf_[vc++] != pos;
        }
        mismatch = mismatch || vc != c || vp != processed;
      }
      cnt_.scan_memo_served.fetch_add(1, std::memory_order_relaxed);
      cnt_.scan_memo_mismatches.fetch_add(mismatch, std::memory_order_relaxed);
    } else if (inline_ok) {
      // Serial path (every cluster below the parallel threshold, and larger
      // ones whose verdicts mostly come from the equivalence cache): plain
      // counters, no std::function call or atomic per node.
      const int64_t t0 = Parallelizer::now_ns();
      if (memo) {  // one allocation for a new template's memo, not a doubling series
        memo->gens.clear();
        memo->ok.clear();
        memo->gens.reserve(static_cast<size_t>(n));
        memo->ok.reserve(static_cast<size_t>(n));
      }
      for (int i = 0; i < n; ++i) {
        int pos = start + i;
        if (pos >= n) pos -= n;
        const NodeInfo& ni = *all[pos];
        bool hit = false;
        const Status* fp = eval_node(pos, ni, fail_buf_[pos], &hit);
        hits += hit;
        ++processed;
        if (memo) {
          memo->gens.push_back(snapshot_.gen[pos]);
          memo->ok.push_back(fp->is_success());
        }
        if (fp->is_success()) {
          found_buf_[c] = &ni;
          found_pos_buf_[c] = pos;
          if (++c == to_find) break;
          continue;
        }
        if (fp->is_unschedulable()) {
          fail_ptr_[pos] = fp;
          continue;
        }
        first_err = *fp;
        has_err = true;
        break;
      }
      if (memo) {
        memo->valid = !has_err && c > 0;
        memo->start = start;
        memo->n = n;
        memo->to_find = to_find;
        memo->epoch = snapshot_.node_epoch;
        memo->processed = processed;
      }
      Parallelizer::record_inline(&filter_site_, Parallelizer::now_ns() - t0, processed, n);
    } else {
      if (memo) memo->valid = false;
      // Forked walk over claimed chunks: a thread keeps its chunk's feasible
      // positions and cache misses in locals and publishes them with one
      // atomic each per chunk (a shared counter bumped per node serialised 16
      // workers on one cache line: the forked walk ran slower than the serial
      // one at 1,024 nodes, profiles/r6/README.md). Feasible nodes are kept in
      // chunk order up to numFeasibleNodesToFind; a chunk in flight when the
      // quota fills finishes its node, the rest of it stops at `stop`.
      std::atomic<int> count{0};
      std::atomic<bool> stop{false};
      std::atomic<uint64_t> amiss{0};
      std::mutex mu;
      parallelizer_->until_forked_ranges(n, [&](int b, int e) {
        constexpr int kLocal = 64;
        int lpos[kLocal];
        int lc = 0;
        uint64_t miss = 0;
        auto flush = [&] {
          if (lc == 0) return;
          const int base = count.fetch_add(lc, std::memory_order_relaxed);
          const int keep = std::min(lc, to_find - base);
          for (int j = 0; j < keep; ++j) {
            found_buf_[base + j] = all[lpos[j]].get();
            found_pos_buf_[base + j] = lpos[j];
          }
          if (base + lc >= to_find) stop.store(true, std::memory_order_relaxed);
          lc = 0;
        };
        for (int i = b; i < e; ++i) {
          if (stop.load(std::memory_order_relaxed)) break;
          int pos = start + i;
          if (pos >= n) pos -= n;
          Status own;
          bool hit = false;
          const Status* fp = eval_node(pos, *all[pos], own, &hit);
          miss += !hit;
          if (fp->is_success()) {
            lpos[lc++] = pos;
            if (lc == kLocal) flush();
            continue;
          }
          if (fp->is_unschedulable()) {
            if (fp == &own) {
              fail_buf_[pos] = std::move(own);
              fp = &fail_buf_[pos];
            }
            fail_ptr_[pos] = fp;
            continue;
          }
          std::lock_guard<std::mutex> g(mu);
          if (!has_err) {
            first_err = *fp;
            has_err = true;
            stop.store(true);
          }
          break;
        }
        flush();
        if (miss) amiss.fetch_add(miss, std::memory_order_relaxed);
      }, &stop, &filter_site_);
      c = std::min(count.load(), to_find);
      // Processed = feasible kept + failed (upstream's feasible +
      // len(NodeToStatusMap)); counted here instead of by a shared atomic
      // that every worker would bump per node.
      processed = c;
      for (int pos = 0; pos < n; ++pos) processed += fail_ptr_[pos] != nullptr;
      hits = static_cast<uint64_t>(std::max<int64_t>(0, static_cast<int64_t>(processed) - static_cast<int64_t>(amiss.load())));
    }
    if (eq_filter) {
      cnt_.eq_filter_hits.fetch_add(hits, std::memory_order_relaxed);
      cnt_.eq_filter_misses.fetch_add(static_cast<uint64_t>(processed) - hits, std::memory_order_relaxed);
    }
    if (has_err) return first_err;
    next_start_node_ = (start + processed) % n;
    feasible.assign(found_buf_.begin(), found_buf_.begin() + c);
    if (feasible_pos) feasible_pos->assign(found_pos_buf_.begin(), found_pos_buf_.begin() + c);
    // Failed nodes mostly share a few Status objects (plugins memoize their
    // failures), so plugins and reasons are tallied per distinct Status first.
    std::vector<std::pair<const Status*, int>> distinct;
    if (feasible.empty() || full_diagnosis) {
      std::unordered_map<const void*, std::unordered_map<const void*, size_t>> index;  // past 32 distinct
      // A fresh diagnosis is recorded in deferred form: (position, status)
      // pairs over the snapshot's names and this cycle's Filter buffers, which
      // outlive every consumer of the diagnosis (PostFilter, FitError).
      const bool fresh = d.node_to_status.empty();
      if (fresh) d.node_to_status.defer(&snapshot_.names, &snapshot_.index);
      else d.node_to_status.reserve(d.node_to_status.size() + static_cast<size_t>(n));
      for (int pos = 0; pos < n; ++pos) {
        const Status* fs = fail_ptr_[pos];
        if (!fs) continue;
        if (fresh) d.node_to_status.append_deferred(pos, fs);
        else d.node_to_status.emplace(snapshot_.names[pos], *fs);
        size_t k = distinct.size();
        if (distinct.size() <= 32) {
          for (size_t j = 0; j < distinct.size(); ++j)
            if (distinct[j].first->reasons_id() == fs->reasons_id() && distinct[j].first->plugin_id() == fs->plugin_id()) {
              k = j;
              break;
            }
        } else {
          auto& by_plugin = index[fs->reasons_id()];
          auto it = by_plugin.find(fs->plugin_id());
          if (it != by_plugin.end()) k = it->second;
        }
        if (k == distinct.size()) {
          distinct.emplace_back(fs, 0);
          if (distinct.size() == 33)  // switch to the index
            for (size_t j = 0; j < distinct.size(); ++j)
              index[distinct[j].first->reasons_id()][distinct[j].first->plugin_id()] = j;
          else if (distinct.size() > 33)
            index[fs->reasons_id()][fs->plugin_id()] = k;
        }
        ++distinct[k].second;
      }
      for (const auto& [s0, cnt] : distinct) d.unschedulable_plugins.insert(s0->failed_plugin());
    }
    if (feasible.empty()) {
      // FitError message: "0/N nodes are available: k reason, ..."
      std::map<std::string, int> reasons;
      for (const auto& [s0, cnt] : distinct)
        for (const auto& r : s0->reasons()) reasons[r] += cnt;
      std::string msg = "0/" + std::to_string(n) + " nodes are available:";
      bool first = true;
      for (const auto& kv : reasons) {
        msg += (first ? " " : ", ") + std::to_string(kv.second) + " " + kv.first;
        first = false;
      }
      msg += ".";
      return Status(Code::Unschedulable, msg);
    }
    if (!ext) return {};
    Status es = run_extender_filters(p, feasible, feasible_pos, d);
    if (!es.is_success() || !feasible.empty()) return es;
    return Status(Code::Unschedulable, fit_error_message(n, d.node_to_status));
  };
  if (rs && !rs->mask.empty()) {
    Status r = walk(rs->mask.data());
    if (!r.is_success() && !r.is_unschedulable()) return r;
    if (!feasible.empty() || !rs->fallback) return r;
    d = Diagnosis{};
    feasible.clear();
    if (feasible_pos) feasible_pos->clear();
  }
  return walk(nullptr);
}

Status Scheduler::filter_listed(Framework& fw, CycleState& s, const Pod& p, Diagnosis& d, NodeList& feasible,
                                EqEntry* eq, const NodeRestriction& rs, std::vector<int>* feasible_pos, bool ext) {
  const auto& all = snapshot_.nodes;
  const int n = static_cast<int>(all.size());
  // The equivalence-cache slot is reused when the verdict is node-local and
  // no nominated pod could change it (the walk's rule, without the
  // per-node nomination signatures).
  const bool use_eq = eq && fw.filters_node_local(p, snapshot_) && !(s.nominated && !s.nominated->empty()) &&
                      !(nominator_ && !nominator_->empty());
  thread_local std::vector<std::pair<int, Status>> failed;
  failed.clear();
  uint64_t hits = 0;
  for (int pos : rs.list) {
    if (pos < 0 || pos >= n) continue;
    const NodeInfo& ni = *all[pos];
    Status st;
    if (use_eq) {
      EqTable& t = eq->table;
      if (t.filter_gen[pos] == snapshot_.gen[pos]) {
        ++hits;
      } else {
        t.filter[pos] = fw.run_filter(s, p, ni);
        t.filter_gen[pos] = snapshot_.gen[pos];
      }
      st = t.filter[pos];
    } else {
      st = fw.run_filter_with_nominated_pods(s, p, ni);
    }
    if (st.is_success()) {
      feasible.push_back(&ni);
      if (feasible_pos) feasible_pos->push_back(pos);
    } else if (st.is_unschedulable()) {
      failed.emplace_back(pos, std::move(st));
    } else {
      return st;
    }
  }
  if (use_eq) {
    cnt_.eq_filter_hits.fetch_add(hits, std::memory_order_relaxed);
    cnt_.eq_filter_misses.fetch_add(rs.list.size() - hits, std::memory_order_relaxed);
  }
  if (!feasible.empty()) {
    if (!ext) return {};
    Status es = run_extender_filters(p, feasible, feasible_pos, d);
    if (!es.is_success() || !feasible.empty()) return es;
  }
  if (rs.fallback) return Status(Code::Unschedulable);  // the caller evaluates every node
  d.node_to_status.reserve(all.size());
  for (int pos = 0; pos < n; ++pos) {
    const Status* st = &rs.excluded;
    for (const auto& [q, fs] : failed)
      if (q == pos) st = &fs;
    d.node_to_status.emplace(snapshot_.names[pos], *st);
  }
  d.unschedulable_plugins.insert(rs.excluded.failed_plugin());
  for (const auto& [q, fs] : failed) d.unschedulable_plugins.insert(fs.failed_plugin());
  return Status(Code::Unschedulable, fit_error_message(n, d.node_to_status));
}

bool Scheduler::extenders_interested(const Pod& p) const {
  for (const auto& e : extenders_)
    if (e->interested(p)) return true;
  return false;
}

Json Scheduler::pod_object(const Pod& p) const {
  if (JsonPtr obj = store_->get("pods", p.ns(), p.name())) return *obj;
  Json md = Json::object();
  md.set("name", Json(p.name()));
  md.set("namespace", Json(p.ns()));
  md.set("uid", Json(p.uid()));
  Json o = Json::object();
  o.set("apiVersion", Json("v1"));
  o.set("kind", Json("Pod"));
  o.set("metadata", std::move(md));
  return o;
}

Status Scheduler::run_extender_filters(const Pod& p, NodeList& feasible, std::vector<int>* pos, Diagnosis& d) {
  Json pod;
  bool have_pod = false;
  ObjectLookup lookup = [this](const std::string& kind, const std::string& ns, const std::string& name) {
    return store_->get(kind, ns, name);
  };
  for (const auto& e : extenders_) {
    if (feasible.empty()) break;
    if (!e->interested(p) || !e->is_filter()) continue;
    if (!have_pod) {
      pod = pod_object(p);
      have_pod = true;
    }
    std::vector<std::string> names;
    names.reserve(feasible.size());
    for (const auto* ni : feasible) names.push_back(ni->name());
    Extender::FilterResult r;
    try {
      r = e->filter(pod, names, lookup);
    } catch (const std::exception& ex) {
      if (e->ignorable()) continue;  // "Skipping extender as it returned error and has ignorable flag set"
      return Status::error(ex.what());
    }
    for (const auto& [node, msg] : r.unresolvable) {
      std::vector<std::string> reasons;
      auto it = d.node_to_status.find(node);
      if (it != d.node_to_status.end()) reasons = it->second.reasons();
      reasons.push_back(msg);
      d.node_to_status[node] = Status(Code::UnschedulableAndUnresolvable, std::move(reasons));
    }
    for (const auto& [node, msg] : r.failed) {
      if (r.unresolvable.count(node)) continue;  // unresolvable takes precedence
      auto it = d.node_to_status.find(node);
      if (it == d.node_to_status.end()) {
        d.node_to_status[node] = Status(Code::Unschedulable, msg);
      } else {
        std::vector<std::string> reasons = it->second.reasons();
        reasons.push_back(msg);
        Status ns(it->second.code(), std::move(reasons));
        if (!it->second.failed_plugin().empty()) ns.with_plugin(it->second.failed_plugin());
        it->second = std::move(ns);
      }
    }
    std::set<std::string> keep(r.nodes.begin(), r.nodes.end());
    size_t w = 0;
    for (size_t i = 0; i < feasible.size(); ++i) {
      if (!keep.count(feasible[i]->name())) continue;
      feasible[w] = feasible[i];
      if (pos) (*pos)[w] = (*pos)[i];
      ++w;
    }
    feasible.resize(w);
    if (pos) pos->resize(w);
  }
  return {};
}

void Scheduler::add_extender_scores(const Pod& p, const NodeList& feasible, std::vector<NodeScore>& scores,
                                    Json* breakdown) {
  std::vector<std::string> names;
  std::unordered_map<std::string, int64_t> combined;
  Json pod;
  bool any = false;
  ObjectLookup lookup = [this](const std::string& kind, const std::string& ns, const std::string& name) {
    return store_->get(kind, ns, name);
  };
  for (const auto& e : extenders_) {
    if (!e->interested(p) || !e->is_prioritizer()) continue;
    if (!any) {
      pod = pod_object(p);
      names.reserve(feasible.size());
      for (const auto* ni : feasible) names.push_back(ni->name());
      any = true;
    }
    try {
      for (const auto& [host, score] : e->prioritize(pod, names, lookup)) {
        combined[host] += score * e->config().weight;
        if (breakdown) {
          Json& node = breakdown->at_or_create(host);
          node.set(e->name(), Json(score));
        }
      }
    } catch (const std::exception&) {
      // "Prioritization errors from extender can be ignored, let k8s/other
      // extenders determine the priorities" (generic_scheduler.go:460-463)
    }
  }
  if (!any) return;
  for (size_t i = 0; i < feasible.size(); ++i) {
    auto it = combined.find(feasible[i]->name());
    if (it != combined.end()) scores[i].score += it->second * (kMaxNodeScore / kMaxExtenderPriority);
  }
}

size_t Scheduler::select_host(const std::vector<NodeScore>& scores) {
  // Uniform among the top-scored nodes, as upstream's reservoir sampling
  // (generic_scheduler.go selectHost), with one draw per cycle instead of one
  // per tie: idle nodes of a large cluster tie by the hundred.
  int64_t best = scores[0].score;
  size_t first = 0;
  uint64_t cnt = 1;
  for (size_t i = 1; i < scores.size(); ++i) {
    if (scores[i].score > best) {
      best = scores[i].score;
      first = i;
      cnt = 1;
    } else if (scores[i].score == best) {
      ++cnt;
    }
  }
  if (cnt == 1) return first;
  uint64_t k = rng_() % cnt;
  for (size_t i = first;; ++i)
    if (scores[i].score == best && k-- == 0) return i;
}

Scheduler::CycleMetrics& Scheduler::cycle_metrics(const Framework& fw) {
  CycleMetrics& m = cycle_metrics_[&fw];
  uint64_t e = metrics_->epoch();
  if (m.epoch != e) {
    static const char* kResults[3] = {"scheduled", "unschedulable", "error"};
    m.algo = &metrics_->histogram("scheduler_scheduling_algorithm_duration_seconds", "");
    m.e2e = &metrics_->histogram("scheduler_e2e_scheduling_duration_seconds", "profile=\"" + fw.profile_name() + "\"");
    for (int i = 0; i < 3; ++i) {
      std::string labels = "profile=\"" + fw.profile_name() + "\",result=\"" + kResults[i] + "\"";
      m.attempt[i] = &metrics_->histogram("scheduler_scheduling_attempt_duration_seconds", labels);
      m.attempts[i] = &metrics_->counter_ref("scheduler_schedule_attempts_total", labels);
    }
    m.epoch = e;
  }
  return m;
}

void Scheduler::schedule_cycle(const QueuedPodInfoPtr& qpi) {
  PodPtr pod = qpi->pod;
  Framework* fw = framework_for(pod->scheduler_name);
  if (!fw) return;
  // skipPodSchedule: deleted or already assumed. The queued object is
  // usually still the lister's current one (no lookup then).
  if (informers_->lists(*pod)) {
    if (pod->terminating() || !pod->node_name.empty()) return;
  } else {
    PodPtr latest = informers_->pod(pod->ns(), pod->name());
    if (!latest || latest->uid() != pod->uid() || latest->terminating() || !latest->node_name.empty()) return;
  }

  int64_t cycle_start = clock_->now_us();
  auto state = std::make_shared<CycleState>();
  state->record_metrics = std::uniform_real_distribution<double>(0, 1)(rng_) < opts_.metrics_sample_rate;
  nom_changed_.clear();
  if (!nominator_->empty()) state->nominated = nominator_->view(&nom_changed_);
  auto to_activate = std::make_shared<PodsToActivate>();
  state->write(kPodsToActivateKey, to_activate);
  int64_t cycle = queue_->scheduling_cycle();
  if (tracer_.enabled())
    tracer_.record(TraceEvent{"queue_wait", pod->key(), "", qpi->timestamp_us, cycle_start - qpi->timestamp_us, 0});

  int64_t lock_wait = 0;
  int64_t snap_start = tracer_.enabled() ? clock_->now_us() : 0;
  bool already_assumed = false;
  int clones = cache_->update_snapshot(snapshot_, tracer_.enabled() ? &lock_wait : nullptr, &pod->uid(), &already_assumed);
  if (already_assumed) return;  // skipPodSchedule: assumed by an earlier cycle
  release_retired();
  refresh_nom_mark(state->nominated.get());
  const std::string& profile = fw->profile_name();
  {
    cnt_.attempts.fetch_add(1, std::memory_order_relaxed);
  }
  int64_t snap_end = clock_->now_us();
  if (tracer_.enabled()) {
    tracer_.record(TraceEvent{"cycle_setup", pod->key(), "", cycle_start, snap_start - cycle_start, 0});
    tracer_.record(TraceEvent{"snapshot", pod->key(),
                              "clones=" + std::to_string(clones) + " lock_wait_us=" + std::to_string(lock_wait),
                              snap_start, snap_end - snap_start, 0});
    tracer_.record(TraceEvent{"snapshot_lock_wait", pod->key(), "", snap_start, lock_wait, 0});
  }

  Diagnosis diag;
  NodeList& feasible = feasible_buf_;
  EqEntry* eq = eq_entry(*fw, *pod);
  Status st = find_nodes_that_fit(*fw, *state, *pod, diag, feasible, eq, false, &feasible_pos_buf_);
  if (tracer_.enabled())
    tracer_.record(TraceEvent{"filter", pod->key(), std::to_string(feasible.size()), snap_end,
                              clock_->now_us() - snap_end, 0});
  std::string host;
  if (st.is_success()) {
    if (feasible.size() == 1) {
      host = feasible[0]->name();
    } else {
      std::vector<NodeScore>& scores = scores_buf_;
      if (!fw->has(kScore)) {
        // No score plugins: every node 1, unless extenders score (then 0 +
        // their priorities, generic_scheduler.go:408-416).
        const bool ext_scores = extenders_interested(*pod);
        scores.assign(feasible.size(), NodeScore{});
        for (auto& sc : scores) sc.score = ext_scores ? 0 : 1;
        st = Status();
      } else {
        st = fw->run_pre_score(*state, *pod, feasible);
        EqScoreCache& esc = esc_buf_;
        esc.local.clear();
        if (eq) fw->local_scorers(*pod, snapshot_, esc.local);
        if (!esc.local.empty()) {
          esc.table = &eq->table;
          esc.pos = feasible_pos_buf_.data();
          esc.npos = feasible.size();
          esc.gen = snapshot_.gen.data();
        }
        if (st.is_success()) st = fw->run_score(*state, *pod, feasible, scores, nullptr, esc.local.empty() ? nullptr : &esc);
      }
      if (st.is_success() && !extenders_.empty()) add_extender_scores(*pod, feasible, scores);
      if (st.is_success()) host = feasible[select_host(scores)]->name();
    }
  }
  int64_t algo_end = clock_->now_us();
  CycleMetrics& cm = cycle_metrics(*fw);
  cm.algo->observe(static_cast<double>(algo_end - cycle_start) / 1e6);
  if (tracer_.enabled())
    tracer_.record(TraceEvent{"schedule", pod->key(), st.is_success() ? host : st.message(), cycle_start,
                              algo_end - cycle_start, 0});

  if (!st.is_success()) {
    std::string nominated;
    bool fit_error = st.is_unschedulable();
    if (fit_error && fw->has(kPostFilter)) {
      auto [res, pst] = fw->run_post_filter(*state, *pod, diag.node_to_status);
      if (pst.is_success()) nominated = res.nominated_node_name;
      {
        cnt_.preemption_attempts.fetch_add(1, std::memory_order_relaxed);
      }
    }
    if (fit_error && !opts_.dump_on_fit_error.empty() && !fit_error_dumped_.exchange(true)) {
      Json d = dump_cache();
      d.set("pod", Json(pod->key()));
      d.set("message", Json(st.message()));
      d.set("at_us", Json(clock_->now_us()));
      if (FILE* f = std::fopen(opts_.dump_on_fit_error.c_str(), "w")) {
        const std::string text = d.dump();
        std::fwrite(text.data(), 1, text.size(), f);
        std::fclose(f);
      }
      if (tracer_.enabled())  // the trace ring up to this failure
        if (FILE* f = std::fopen((opts_.dump_on_fit_error + ".trace.json").c_str(), "w")) {
          const std::string text = tracer_.chrome_json();
          std::fwrite(text.data(), 1, text.size(), f);
          std::fclose(f);
        }
    }
    const int result = fit_error ? 1 : 2;
    cm.attempts[result]->inc();
    cm.attempt[result]->observe(static_cast<double>(clock_->now_us() - cycle_start) / 1e6);
    {
      (fit_error ? cnt_.unschedulable : cnt_.errors).fetch_add(1, std::memory_order_relaxed);
    }
    handle_failure(*fw, qpi, st, fit_error ? "Unschedulable" : "SchedulerError", nominated, cycle,
                   diag.unschedulable_plugins);
    return;
  }

  // Assume.
  auto assumed = std::make_shared<Pod>(*pod);
  assumed->node_name = host;
  Status ast = cache_->assume_pod(assumed);
  if (!ast.is_success()) {
    handle_failure(*fw, qpi, ast, "SchedulerError", "", cycle, {});
    return;
  }
  // An assumed pod is accounted on its node; drop its nomination so it is not
  // counted twice by nominated-pod-aware checks (scheduler.go assume():
  // DeleteNominatedPodIfExists).
  if (!nominator_->empty()) nominator_->remove(*assumed);
  int64_t t_assumed = tracer_.enabled() ? clock_->now_us() : 0;
  // Reserve.
  Status rst = fw->run_reserve(*state, assumed, host);
  int64_t t_reserved = tracer_.enabled() ? clock_->now_us() : 0;
  if (!rst.is_success()) {
    fw->run_unreserve(*state, assumed, host);
    cache_->forget_pod(*assumed);
    cnt_.errors.fetch_add(1, std::memory_order_relaxed);
    handle_failure(*fw, qpi, rst, rst.is_unschedulable() ? "Unschedulable" : "SchedulerError", "", cycle,
                   rst.failed_plugin().empty() ? std::set<std::string>{} : std::set<std::string>{rst.failed_plugin()});
    return;
  }
  // Permit.
  int64_t permit_start = clock_->now_us();
  inflight_.fetch_add(1);
  auto task = std::make_shared<BindTask>();
  task->self = this;
  task->fw = fw;
  task->state = state;
  task->qpi = qpi;
  task->assumed = assumed;
  task->host = host;
  task->cycle = cycle;
  task->permit_start_us = permit_start;
  task->to_activate = to_activate;
  task->e2e = cycle_metrics(*fw).e2e;
  task->keep = task;
  BindTask* tp = task.get();
  // The binding cycles this Permit releases (the gang's waiting members and
  // this pod) reach the binder pool in one hand-over.
  std::optional<Executor::Batch> batch(std::in_place, *binder_);
  Status pst = fw->run_permit(*state, assumed, host, [tp](const Status& wst) {
    tp->permit_status = wst;
    tp->self->binder_->submit([tp] { run_bind_task(tp); });
  });
  if (!pst.is_success() && !pst.is_wait()) {
    task->keep.reset();  // rejected before waiting: the callback never runs
    inflight_.fetch_sub(1);
    fw->run_unreserve(*state, assumed, host);
    cache_->forget_pod(*assumed);
    {
      cnt_.unschedulable.fetch_add(1, std::memory_order_relaxed);
    }
    handle_failure(*fw, qpi, pst, pst.is_unschedulable() ? "Unschedulable" : "SchedulerError", "", cycle,
                   pst.failed_plugin().empty() ? std::set<std::string>{} : std::set<std::string>{pst.failed_plugin()});
    return;
  }
  int64_t t_permitted = tracer_.enabled() ? clock_->now_us() : 0;
  if (pst.is_success()) note_gang_event(*assumed, false);
  // Activate siblings stashed by plugins (scheduler.go:543-548).
  {
    std::vector<PodPtr> act;
    {
      std::lock_guard<std::mutex> g(to_activate->mu);
      act.swap(to_activate->pods);
    }
    if (!act.empty()) queue_->activate(act);
  }
  cm.attempts[0]->inc();
  cm.attempt[0]->observe(static_cast<double>(clock_->now_us() - cycle_start) / 1e6);
  {
    cnt_.scheduled.fetch_add(1, std::memory_order_relaxed);
  }
  if (pst.is_success()) binder_->submit([tp] { run_bind_task(tp); });
  batch.reset();
  if (tracer_.enabled()) {
    int64_t t_end = clock_->now_us();
    tracer_.record(TraceEvent{"assume_reserve_permit", assumed->key(), "", algo_end, t_end - algo_end, 0});
    tracer_.record(TraceEvent{"assume", assumed->key(), "", algo_end, t_assumed - algo_end, 0});
    tracer_.record(TraceEvent{"reserve", assumed->key(), "", t_assumed, t_reserved - t_assumed, 0});
    tracer_.record(TraceEvent{"permit", assumed->key(), "", t_reserved, t_permitted - t_reserved, 0});
    tracer_.record(TraceEvent{"activate_metrics", assumed->key(), "", t_permitted, t_end - t_permitted, 0});
  }
}

namespace {
// Polls `done` every 20 us until it holds or `timeout_us` passes (wall time,
// not clock_: a fake clock in tests does not advance). No spinning: the
// waiter shares its CPU domain with the scheduler's threads.
template <class F>
bool poll_until(F done, int64_t timeout_us) {
  const auto end = std::chrono::steady_clock::now() + std::chrono::microseconds(timeout_us);
  while (!done()) {
    if (std::chrono::steady_clock::now() > end) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  return true;
}
}  // namespace

bool Scheduler::wait_bound(uint64_t target, int64_t timeout_us) const {
  // Polls a counter instead of a condition variable: the binder threads
  // then pay nothing per bind.
  return poll_until([&] { return bound_total_.load(std::memory_order_acquire) >= target; }, timeout_us);
}

bool Scheduler::wait_cache_empty(int64_t timeout_us) const {
  return poll_until([&] { return cache_->pod_count() == 0; }, timeout_us);
}

Json Scheduler::check_cache() const {
  // The listers and the cache are read one after the other, not atomically:
  // an informer event landing between the two reads shows as a difference
  // that the next read no longer has. Such a difference is read again (up to
  // ~50 ms); one that persists is reported. `reads` says how many it took.
  Json out;
  int reads = 0;
  for (; reads < 25; ++reads) {
    if (reads) std::this_thread::sleep_for(std::chrono::milliseconds(2));
    std::vector<PodPtr> assigned;
    for (auto& p : informers_->all_pods())
      if (!p->node_name.empty()) assigned.push_back(std::move(p));
    std::vector<std::string> nodes;
    for (const auto& n : store_->list("nodes", "")) nodes.push_back((*n)["metadata"]["name"].as_string());
    out = cache_->check(assigned, nodes);
    if (out["clean"].as_bool()) break;
  }
  out.set("reads", Json(static_cast<int64_t>(std::min(reads + 1, 25))));
  return out;
}

Json Scheduler::dump_cache() const {
  Json out = cache_->dump();
  auto c = queue_->counts();
  Json q = Json::object();
  q.set("active", Json(static_cast<int64_t>(c.active)));
  q.set("backoff", Json(static_cast<int64_t>(c.backoff)));
  q.set("unschedulable", Json(static_cast<int64_t>(c.unschedulable)));
  Json pending = Json::array();
  for (const auto& qpi : queue_->pending_pods()) pending.push_back(Json(qpi->pod->key()));
  q.set("pods", std::move(pending));
  out.set("queue", std::move(q));
  int64_t waiting = 0;
  for (const auto& w : waiting_) waiting += static_cast<int64_t>(w->size());
  out.set("waiting_pods", Json(waiting));
  out.set("nominated_pods", Json(static_cast<int64_t>(nominator_->size())));
  return out;
}

namespace {
Code code_from_name(const std::string& n) {
  for (Code c : {Code::Success, Code::Error, Code::Unschedulable, Code::UnschedulableAndUnresolvable, Code::Wait,
                 Code::Skip})
    if (n == code_name(c)) return c;
  throw std::runtime_error("unknown status code " + n);
}
Json status_json(const Status& st) {
  Json out = Json::object();
  out.set("code", Json(code_name(st.code())));
  out.set("message", Json(st.message()));
  return out;
}
}  // namespace

Json Scheduler::plugin_call(const std::string& plugin, const std::string& point, const Json& args) {
  std::lock_guard<std::mutex> g(sched_mu_);
  Framework* fw = frameworks_.front().get();
  if (args["schedulerName"].is_string()) fw = framework_for(args["schedulerName"].as_string());
  if (!fw) throw std::runtime_error("no such profile");
  Plugin* pl = nullptr;
  for (const auto& x : fw->all_plugins())
    if (x->name() == plugin) pl = x.get();
  if (!pl) throw std::runtime_error("plugin " + plugin + " is not enabled in the profile");
  cache_->update_snapshot(snapshot_);
  auto state = std::make_shared<CycleState>();
  state->write(kPodsToActivateKey, std::make_shared<PodsToActivate>());
  auto parse = [&](const Json& j) {
    auto p = Pod::from_json(j, *gpu_names_);
    if (p->uid().empty()) p->meta.uid = "harness-" + p->key();
    return p;
  };
  PodPtr pod = args.get("pod") ? parse(args["pod"]) : nullptr;
  const std::string node = args["node"].str_or("");
  if (point == "less") {
    QueuedPodInfo a, b;
    a.pod = parse(args["a"]);
    b.pod = parse(args["b"]);
    a.initial_attempt_wall = args["a_initial_attempt_us"].as_int(0);
    b.initial_attempt_wall = args["b_initial_attempt_us"].as_int(0);
    Json out = Json::object();
    out.set("less", Json(pl->less(a, b)));
    return out;
  }
  if (!pod) throw std::runtime_error("args.pod is required");
  if (point == "preFilter") return status_json(pl->pre_filter(*state, *pod));
  if (point == "postFilter") {
    NodeStatusMap m;
    for (const auto& [n, c] : args["statuses"].members()) {
      Status st(code_from_name(c.as_string()), c.as_string() == "Success" ? "" : "harness");
      m.emplace(n, st);
    }
    auto [res, st] = pl->post_filter(*state, *pod, m);
    Json out = status_json(st);
    out.set("nominatedNodeName", Json(res.nominated_node_name));
    return out;
  }
  if (point == "permit" || point == "reserve" || point == "unreserve" || point == "postBind") {
    // As in the real cycle these run on the assumed pod: the cache holds it
    // (Coscheduling's assigned count includes it) while the point runs.
    auto assumed = std::make_shared<Pod>(*pod);
    assumed->node_name = node;
    const bool assume = !node.empty() && args["assume"].as_bool(true) && point != "postBind";
    if (assume) {
      Status ast = cache_->assume_pod(assumed);
      if (!ast.is_success()) return status_json(ast);
    }
    Json out;
    if (point == "permit") {
      auto [st, timeout] = pl->permit(*state, assumed, node);
      out = status_json(st);
      out.set("timeout_us", Json(timeout));
    } else if (point == "reserve") {
      out = status_json(pl->reserve(*state, assumed, node));
    } else if (point == "unreserve") {
      pl->unreserve(*state, assumed, node);
      out = status_json(Status());
    } else {
      pl->post_bind(*state, assumed, node);
      out = status_json(Status());
    }
    if (assume) cache_->forget_pod(*assumed);
    return out;
  }
  if (point == "filter" || point == "score") {
    // One plugin's Filter verdicts / Score+NormalizeScore over the snapshot's
    // nodes (or args.nodes, in that order), as the reference's plugin unit
    // tests call them (after the plugin's own PreFilter / PreScore).
    NodeList nodes;
    if (args["nodes"].is_array()) {
      for (const auto& n : args["nodes"].items()) {
        auto it = snapshot_.index.find(n.as_string());
        if (it == snapshot_.index.end()) throw std::runtime_error("no node " + n.as_string());
        nodes.push_back(snapshot_.nodes[it->second].get());
      }
    } else {
      for (const auto& ni : snapshot_.nodes) nodes.push_back(ni.get());
    }
    Json out = Json::object();
    if (point == "filter") {
      if (pl->points() & kPreFilter) {
        Status pst = pl->pre_filter(*state, *pod);
        if (!pst.is_success()) {
          out.set("preFilter", status_json(pst));
          return out;
        }
      }
      Json per = Json::object();
      for (const NodeInfo* ni : nodes) per.set(ni->name(), status_json(pl->filter(*state, *pod, *ni)));
      out.set("nodes", std::move(per));
      return out;
    }
    if (pl->points() & kPreScore) {
      Status pst = pl->pre_score(*state, *pod, nodes);
      if (!pst.is_success()) {
        out.set("preScore", status_json(pst));
        return out;
      }
    }
    std::vector<NodeScore> scores(nodes.size());
    Json raw = Json::object();
    for (size_t i = 0; i < nodes.size(); ++i) {
      auto [sc, st] = pl->score(*state, *pod, *nodes[i]);
      if (!st.is_success()) throw std::runtime_error("score " + nodes[i]->name() + ": " + st.message());
      scores[i].name = &nodes[i]->name();
      scores[i].score = sc;
      raw.set(nodes[i]->name(), Json(sc));
    }
    if (pl->has_normalize_score()) {
      Status nst = pl->normalize_score(*state, *pod, scores);
      if (!nst.is_success()) throw std::runtime_error("normalize: " + nst.message());
    }
    Json norm = Json::object();
    for (size_t i = 0; i < nodes.size(); ++i) norm.set(nodes[i]->name(), Json(scores[i].score));
    out.set("raw", std::move(raw));
    out.set("scores", std::move(norm));
    return out;
  }
  if (args["runPreFilter"].as_bool(false)) {
    Status st = fw->run_pre_filter(*state, *pod);
    if (!st.is_success()) return status_json(st);
  }
  return pl->debug_call(point, *state, pod, args);
}

Json Scheduler::explain(const Json& pod_obj) {
  std::lock_guard<std::mutex> g(sched_mu_);
  Json out = Json::object();
  auto pod = Pod::from_json(pod_obj, *gpu_names_);
  Framework* fw = framework_for(pod->scheduler_name);
  if (!fw) {
    out.set("error", Json("no profile for schedulerName " + pod->scheduler_name.str()));
    return out;
  }
  if (pod->uid().empty()) pod->meta.uid = "explain-" + pod->key();
  cache_->update_snapshot(snapshot_);
  auto state = std::make_shared<CycleState>();
  state->write(kPodsToActivateKey, std::make_shared<PodsToActivate>());
  Diagnosis d;
  NodeList feasible;
  int saved_start = next_start_node_;
  Status st = find_nodes_that_fit(*fw, *state, *pod, d, feasible, nullptr, true);
  next_start_node_ = saved_start;
  out.set("code", Json(code_name(st.code())));
  out.set("message", Json(st.message()));
  Json filt = Json::object();
  for (const auto& [node, s] : d.node_to_status) {
    Json e = Json::object();
    e.set("plugin", Json(s.failed_plugin()));
    e.set("reason", Json(s.message()));
    e.set("code", Json(code_name(s.code())));
    filt.set(node, std::move(e));
  }
  out.set("filtered", std::move(filt));
  Json feas = Json::array();
  for (const auto& ni : feasible) feas.push_back(Json(ni->name()));
  out.set("feasible", std::move(feas));
  if (st.is_success() && !feasible.empty() && fw->has(kScore)) {
    std::vector<NodeScore> scores;
    Framework::ScoreBreakdown bd;
    Status ps = fw->run_pre_score(*state, *pod, feasible);
    if (ps.is_success()) ps = fw->run_score(*state, *pod, feasible, scores, &bd);
    if (ps.is_success()) {
      Json ext = Json::object();
      if (!extenders_.empty()) add_extender_scores(*pod, feasible, scores, &ext);
      Json sc = Json::object();
      for (size_t i = 0; i < feasible.size(); ++i) {
        Json node = Json::object();
        for (const auto& [plugin, vals] : bd) node.set(plugin, Json(vals[i]));
        if (const Json* e = ext.get(feasible[i]->name())) node.set("extenders", *e);
        node.set("total", Json(scores[i].score));
        sc.set(feasible[i]->name(), std::move(node));
      }
      out.set("scores", std::move(sc));
      out.set("selected", Json(feasible[select_host(scores)]->name()));
      // The scheduling path's totals (all-zero plugins skipped, their
      // normalized constant still added, the plugins' snapshot-array paths
      // given the nodes' positions) for parity checks against "total".
      // The template's equivalence slots are used as the scheduling cycle
      // uses them (hits included), so the parity check covers cached sums.
      std::vector<NodeScore> hot;
      EqScoreCache hot_cache;
      std::vector<int> hot_pos;
      EqEntry* eq = eq_entry(*fw, *pod);
      if (eq) fw->local_scorers(*pod, snapshot_, hot_cache.local);
      for (const NodeInfo* ni : feasible) {
        auto it = snapshot_.index.find(ni->name());
        if (it == snapshot_.index.end()) break;
        hot_pos.push_back(static_cast<int>(it->second));
      }
      if (eq && !hot_cache.local.empty()) hot_cache.table = &eq->table;
      hot_cache.pos = hot_pos.data();
      hot_cache.npos = hot_pos.size();
      hot_cache.gen = snapshot_.gen.data();
      EqScoreCache* hot_eq = hot_pos.size() == feasible.size() ? &hot_cache : nullptr;
      if (fw->run_score(*state, *pod, feasible, hot, nullptr, hot_eq).is_success()) {
        Json h = Json::object();
        for (size_t i = 0; i < feasible.size(); ++i) h.set(feasible[i]->name(), Json(hot[i].score));
        out.set("hot_path_totals", std::move(h));
      }
    } else {
      out.set("score_error", Json(ps.message()));
    }
  } else if (feasible.size() == 1) {
    out.set("selected", Json(feasible[0]->name()));
  }
  return out;
}

double Scheduler::score_benchmark(const Json& pod_obj, int iterations, Json* out) {
  std::lock_guard<std::mutex> g(sched_mu_);
  auto pod = Pod::from_json(pod_obj, *gpu_names_);
  Framework* fw = framework_for(pod->scheduler_name);
  if (!fw) throw std::runtime_error("no profile for schedulerName " + pod->scheduler_name.str());
  cache_->update_snapshot(snapshot_);
  NodeList nodes;
  nodes.reserve(snapshot_.nodes.size());
  for (const auto& ni : snapshot_.nodes) nodes.push_back(ni.get());
  int64_t checksum = 0;
  int64_t t0 = clock_->now_us();
  for (int it = 0; it < std::max(1, iterations); ++it) {
    CycleState st;
    std::vector<NodeScore> scores;
    Status s = fw->run_pre_score(st, *pod, nodes);
    if (s.is_success()) s = fw->run_score(st, *pod, nodes, scores);
    if (!s.is_success()) throw std::runtime_error(s.message());
    for (const auto& x : scores) checksum += x.score;
  }
  double us = static_cast<double>(clock_->now_us() - t0) / std::max(1, iterations);
  if (out) {
    *out = Json::object();
    out->set("nodes", Json(static_cast<int64_t>(nodes.size())));
    out->set("us_per_pass", Json(us));
    out->set("checksum", Json(checksum));
  }
  return us;
}

Scheduler::BindMetrics& Scheduler::bind_metrics() {
  BindMetrics& m = bind_metrics_;
  uint64_t e = metrics_->epoch();
  if (m.epoch.load(std::memory_order_acquire) == e) return m;
  std::lock_guard<std::mutex> g(bind_metrics_mu_);
  if (m.epoch.load(std::memory_order_acquire) == e) return m;
  m.binding.store(&metrics_->histogram("xsched_binding_duration_seconds", ""));
  m.attempts.store(&metrics_->histogram("scheduler_pod_scheduling_attempts", ""));
  m.permit_wait[0].store(&metrics_->histogram("scheduler_permit_wait_duration_seconds", "result=\"Success\""));
  m.permit_wait[1].store(&metrics_->histogram("scheduler_permit_wait_duration_seconds", "result=\"Unschedulable\""));
  for (int a = 1; a <= 8; ++a)
    m.pod_duration[a - 1].store(
        &metrics_->histogram("scheduler_pod_scheduling_duration_seconds", "attempts=\"" + std::to_string(a) + "\""));
  m.epoch.store(e, std::memory_order_release);
  return m;
}

void Scheduler::binding_cycle(const BindTask& t, const Status& permit_status) {
  Framework* fw = t.fw;
  const CycleStatePtr& s = t.state;
  const QueuedPodInfoPtr& qpi = t.qpi;
  const PodPtr& assumed = t.assumed;
  const std::string& host = t.host;
  const int64_t cycle = t.cycle, wait_start_us = t.permit_start_us;
  const std::shared_ptr<PodsToActivate>& to_activate = t.to_activate;
  int64_t t0 = clock_->now_us();
  auto fail = [&](const Status& st, const std::string& reason) {
    fw->run_unreserve(*s, assumed, host);
    cache_->forget_pod(*assumed);
    // A forgotten pod frees resources: let waiting pods retry (AssignedPodDelete).
    queue_->move_all_to_active_or_backoff(ClusterEvent{"Pod", kDelete, "AssignedPodDelete"});
    capacity_freed();
    {
      cnt_.bind_failures.fetch_add(1, std::memory_order_relaxed);
    }
    handle_failure(*fw, qpi, st, reason, "", cycle,
                   st.failed_plugin().empty() ? std::set<std::string>{} : std::set<std::string>{st.failed_plugin()});
    inflight_.fetch_sub(1);
  };
  BindMetrics& bm = bind_metrics();
  if (wait_start_us > 0 && t0 - wait_start_us > 0) {
    bm.permit_wait[permit_status.is_success() ? 0 : 1].load(std::memory_order_relaxed)
        ->observe(static_cast<double>(t0 - wait_start_us) / 1e6);
    if (tracer_.enabled())
      tracer_.record(TraceEvent{"permit_wait", assumed->key(), code_name(permit_status.code()), wait_start_us,
                                t0 - wait_start_us, 1});
  }
  if (!permit_status.is_success()) {
    fail(permit_status, permit_status.is_unschedulable() ? "Unschedulable" : "SchedulerError");
    return;
  }
  Status st = fw->run_pre_bind(*s, assumed, host);
  if (!st.is_success()) {
    fail(st, "SchedulerError");
    return;
  }
  // extendersBinding (scheduler.go bind()): the first interested binder
  // extender binds instead of the Bind plugins.
  Extender* binder = nullptr;
  for (const auto& e : extenders_)
    if (e->is_binder() && e->interested(*assumed)) {
      binder = e.get();
      break;
    }
  if (binder) {
    try {
      binder->bind(assumed->ns(), assumed->name(), assumed->uid(), host);
      st = Status();
    } catch (const std::exception& ex) {
      st = Status::error(std::string("extender ") + binder->name() + " bind: " + ex.what());
    }
  } else {
    st = fw->run_bind(*s, assumed, host);
  }
  if (st.is_skip()) st = Status(Code::Error, "no bind plugin bound the pod");
  if (!st.is_success()) {
    fail(st, "SchedulerError");
    return;
  }
  cache_->finish_binding(*assumed);
  int64_t t1 = clock_->now_us();
  bm.binding.load(std::memory_order_relaxed)->observe(static_cast<double>(t1 - t0) / 1e6);
  t.e2e->observe(static_cast<double>(t1 - qpi->timestamp_us) / 1e6);
  Histogram* pd = qpi->attempts >= 1 && qpi->attempts <= 8
                      ? bm.pod_duration[qpi->attempts - 1].load(std::memory_order_relaxed)
                      : &metrics_->histogram("scheduler_pod_scheduling_duration_seconds",
                                             "attempts=\"" + std::to_string(qpi->attempts) + "\"");
  pd->observe(static_cast<double>(t1 - qpi->initial_attempt_us) / 1e6);
  bm.attempts.load(std::memory_order_relaxed)->observe(qpi->attempts);
  if (tracer_.enabled()) tracer_.record(TraceEvent{"bind", assumed->key(), host, t0, t1 - t0, 1});
  fw->run_post_bind(*s, assumed, host);
  if (tracer_.enabled()) {
    const int64_t t2 = clock_->now_us();
    tracer_.record(TraceEvent{"post_bind", assumed->key(), "", t1, t2 - t1, 1});
  }
  {
    cnt_.bound.fetch_add(1, std::memory_order_relaxed);
  }
  bound_total_.fetch_add(1, std::memory_order_release);
  note_gang_event(*assumed, true);
  {
    std::vector<PodPtr> act;
    {
      std::lock_guard<std::mutex> g(to_activate->mu);
      act.swap(to_activate->pods);
    }
    if (!act.empty()) queue_->activate(act);
  }
  inflight_.fetch_sub(1);
}

void Scheduler::handle_failure(Framework& fw, const QueuedPodInfoPtr& qpi, const Status& st, const std::string& reason,
                               const std::string& nominated, int64_t cycle, const std::set<std::string>& plugins) {
  PodPtr pod = qpi->pod;
  // updatePod is skipped when the condition and nomination are unchanged
  // since this pod's last failure (remembered on its queue entry, so the
  // memo lives and dies with the pod: no scheduler-wide map to sweep).
  std::string condition = st.message() + "|" + nominated;
  const bool same_condition = qpi->last_condition == condition && nominated == pod->nominated_node_name;
  // Requeue the latest version unless it was deleted or got assigned.
  PodPtr latest = informers_->pod(pod->ns(), pod->name());
  if (latest && latest->uid() == pod->uid() && latest->node_name.empty() && !latest->terminating()) {
    auto nq = std::make_shared<QueuedPodInfo>(*qpi);
    nq->pod = latest;
    nq->unschedulable_plugins = plugins;
    nq->last_condition = condition;
    queue_->add_unschedulable_if_not_present(nq, cycle);
  }
  // After the requeue (which re-registers the pod's *observed* nomination):
  // the next cycle must already see this one, before the status patch comes
  // back through the informer (scheduler.go handleSchedulingFailure).
  if (!nominated.empty()) nominator_->add(latest && latest->uid() == pod->uid() ? latest : pod, nominated);
  // The event goes out on the status writer (kube-scheduler's recorder is
  // asynchronous too); the status update stays on the scheduling loop, as
  // upstream's updatePod: written asynchronously it could land after a later
  // cycle bound the pod and overwrite its PodScheduled=True condition. (Moved
  // to the status writer with a resourceVersion precondition, it cost open-loop
  // capacity on the box: parked gangs at 112k pods/s went from 44-86 to 1,917,
  // profiles/r6/README.md, r6x. The inline patch is backpressure.)
  ApiClient* client = fw.handle().client;
  status_writer_->submit([client, pod, msg = st.message()] {
    try {
      client->record_event("Pod", pod->ns(), pod->name(), "Warning", "FailedScheduling", msg);
    } catch (const std::exception&) {
    }
  });
  if (!opts_.status_updates || same_condition) return;
  // updatePod: PodScheduled=False condition + nominatedNodeName, only when changed.
  std::string msg = st.message();
  Json patch = Json::object();
  Json status = Json::object();
  Json cond = Json::object();
  cond.set("type", Json("PodScheduled"));
  cond.set("status", Json("False"));
  cond.set("reason", Json(reason));
  cond.set("message", Json(msg));
  Json conds = Json::array();
  conds.push_back(std::move(cond));
  status.set("conditions", std::move(conds));
  if (!nominated.empty()) status.set("nominatedNodeName", Json(nominated));
  patch.set("status", std::move(status));
  try {
    client->patch("pods", pod->ns(), pod->name(), patch);
  } catch (const std::exception&) {
  }
}

}  // namespace xsched
