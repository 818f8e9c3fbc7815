// Native driver: replays benchmark waves against the C++ store + scheduler
// without Python. Used for (a) ThreadSanitizer runs of the concurrent core
// (build_ext --tsan) and (b) profiling the scheduling cycle.
//
//   xsched_stress <dir> [waves]
// <dir> holds nodes.json, nrts.json, config.json (native profile config) and
// wave_<i>.json files {"podgroups":[...],"pods":[...]} written by
// flex_gpu_scheduler_amd/tools/stress.py, and optionally init.json (pods
// created and bound before every wave, untimed: e.g. PreemptionBasic's
// low-priority victims).
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <filesystem>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>

#include "apiserver/apiserver.h"
#include "common/alloc.h"
#include "rest/kube.h"
#include "scheduler/openloop.h"
#include "scheduler/scheduler.h"
#include "tools/sampler.h"

using namespace xsched;

static std::string slurp(const std::string& p) {
  std::ifstream f(p);
  if (!f) {
    std::fprintf(stderr, "cannot read %s\n", p.c_str());
    std::exit(2);
  }
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

// `xsched_stress apiserver [clients] [objects]`: the native HTTP API server
// under concurrent REST clients (create / get / patch / list with selectors /
// bind / delete), two raw watch streams and a LIST/WATCH mirror, then a stop
// with streams still open: the sanitizer builds run this for the server's
// connection threads, watcher registry and shutdown.
static int apiserver_stress(int clients, int objects) {
  auto store = std::make_shared<ObjectStore>();
  store->create("nodes", Json::parse(R"({"metadata":{"name":"n0"},"status":{"allocatable":{"cpu":"64","pods":"1000"}}})"));
  apiserver::Options o;
  apiserver::Server srv(store, o);
  srv.start();
  rest::Endpoint ep;
  ep.port = srv.port();
  auto local = std::make_shared<ObjectStore>();
  rest::RemoteMirror mirror(ep, local, {"pods", "nodes"});
  mirror.start();
  if (!mirror.wait_synced(10'000)) {
    std::fprintf(stderr, "mirror did not sync\n");
    return 1;
  }
  std::atomic<int> failures{0};
  std::atomic<uint64_t> requests{0};
  std::atomic<bool> stop_watch{false};
  std::vector<std::thread> watchers;
  std::atomic<uint64_t> watch_lines{0};
  for (int w = 0; w < 2; ++w) {
    watchers.emplace_back([&] {
      try {
        rest::HttpConn c(ep, nullptr, true);
        if (c.open_stream("/api/v1/pods?watch=1&allowWatchBookmarks=true") != 200) {
          ++failures;
          return;
        }
        std::string line;
        while (!stop_watch.load() && c.next_line(line)) ++watch_lines;
      } catch (const std::exception&) {
      }
    });
  }
  std::vector<std::thread> ts;
  for (int t = 0; t < clients; ++t) {
    ts.emplace_back([&, t] {
      rest::ConnPool pool(ep);
      auto call = [&](const char* m, const std::string& path, const std::string& body, int want,
                      const char* ct = "application/json") {
        auto r = pool.call(m, path, body, ct);
        ++requests;
        if (r.status != want) {
          ++failures;
          std::fprintf(stderr, "%s %s -> %d %s\n", m, path.c_str(), r.status, r.body.substr(0, 200).c_str());
        }
      };
      for (int i = 0; i < objects; ++i) {
        std::string name = "p" + std::to_string(t) + "-" + std::to_string(i);
        std::string path = "/api/v1/namespaces/s/pods/" + name;
        call("POST", "/api/v1/namespaces/s/pods",
             R"({"metadata":{"name":")" + name + R"(","labels":{"t":")" + std::to_string(t) +
                 R"("}},"spec":{"containers":[{"name":"c"}]}})",
             201);
        call("GET", path, "", 200);
        call("PATCH", path, R"({"metadata":{"annotations":{"k":"v"}}})", 200, "application/merge-patch+json");
        call("PATCH", path, R"([{"op":"add","path":"/metadata/labels/j","value":"x"}])", 200,
             "application/json-patch+json");
        call("GET", "/api/v1/namespaces/s/pods?labelSelector=t%3D" + std::to_string(t) + "%2Cj", "", 200);
        call("POST", path + "/binding", R"({"target":{"name":"n0"}})", 201);
        call("DELETE", path, "", 200);
        call("GET", path, "", 404);
      }
    });
  }
  for (auto& t : ts) t.join();
  for (int i = 0; i < 500 && local->count("pods") > 0; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(10));
  size_t left = local->count("pods");
  // Stop with both watch streams still open: the server must end them.
  srv.stop();
  stop_watch = true;
  for (auto& w : watchers) w.join();
  mirror.stop();
  std::printf("apiserver stress: %llu requests, %d failures, %llu watch lines, %zu pods left in the mirror\n",
              static_cast<unsigned long long>(requests.load()), failures.load(),
              static_cast<unsigned long long>(watch_lines.load()), left);
  return failures.load() == 0 && left == 0 ? 0 : 1;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <dir> [waves] | apiserver [clients] [objects]\n", argv[0]);
    return 2;
  }
  tune_allocator();  // XSCHED_MALLOC_TUNE=0 keeps glibc's defaults (A/B runs)
  if (std::string(argv[1]) == "apiserver")
    return apiserver_stress(argc > 2 ? std::atoi(argv[2]) : 8, argc > 3 ? std::atoi(argv[3]) : 200);
  std::string dir = argv[1];
  int waves = argc > 2 ? std::atoi(argv[2]) : 4;
  auto store = std::make_shared<ObjectStore>();
  auto load_many = [&](const std::string& kind, const std::string& file) {
    Json arr = Json::parse(slurp(dir + "/" + file));
    std::vector<Json> v(arr.items().begin(), arr.items().end());
    store->create_many(kind, std::move(v));
  };
  load_many("nodes", "nodes.json");
  load_many("noderesourcetopologies", "nrts.json");
  // extra.json: {"<kind>": [objects]} created before the scheduler starts
  // (e.g. a scheduler_perf workload's ElasticQuotas).
  if (std::filesystem::exists(dir + "/extra.json")) {
    Json extra = Json::parse(slurp(dir + "/extra.json"));
    for (const auto& [kind, objs] : extra.members()) {
      std::vector<Json> v(objs.items().begin(), objs.items().end());
      store->create_many(kind, std::move(v));
    }
  }
  Json cfg = Json::parse(slurp(dir + "/config.json"));
  Scheduler sched(store, cfg);
  sched.start();
  // XSCHED_SAMPLE=<file>: CPU-sample every thread during the waves
  // (tools/sample_report.py symbolizes the dump).
  const char* sample_path = std::getenv("XSCHED_SAMPLE");
  if (sample_path) sampler::start(std::getenv("XSCHED_SAMPLE_HZ") ? std::atoi(std::getenv("XSCHED_SAMPLE_HZ")) : 4000);
  // Open-loop mode: <dir>/openloop.json {"gangs":[{"podgroup":..,"pods":[..]}],
  // "offsets_us":[..], "hold_us":N} written by tools/stress.py --openloop RATE
  // (utils/openloop.py plan()); arrivals paced by run_open_loop.
  if (std::filesystem::exists(dir + "/openloop.json")) {
    Json ol = Json::parse(slurp(dir + "/openloop.json"));
    std::vector<OpenLoopGang> gangs;
    for (const auto& g : ol["gangs"].items()) {
      OpenLoopGang og;
      og.pod_group = g["podgroup"];
      og.pods.assign(g["pods"].items().begin(), g["pods"].items().end());
      gangs.push_back(std::move(og));
    }
    std::vector<int64_t> offsets;
    for (const auto& o : ol["offsets_us"].items()) offsets.push_back(o.as_int());
    size_t pods = 0;
    for (const auto& g : gangs) pods += g.pods.size();
    OpenLoopResult r = run_open_loop(*store, sched, std::move(gangs), offsets, ol["hold_us"].as_int(1000), 10'000'000);
    if (sample_path) sampler::dump(sample_path);
    size_t unbound = 0;
    for (const auto& g : r.gangs) unbound += g.bound_us == 0;
    sched.stop();
    std::printf("openloop: %zu pods, %zu gangs unbound, wall %.4fs (%.0f pods/s), mean arrival lag %.1f us\n", pods,
                unbound, r.wall_us / 1e6, pods / (r.wall_us / 1e6), r.gangs.empty() ? 0.0 : double(r.late_us) / r.gangs.size());
    return unbound ? 1 : 0;
  }
  uint64_t bound = 0;
  double total_s = 0;
  size_t total_pods = 0;
  const bool has_init = std::filesystem::exists(dir + "/init.json");
  auto wait_bound = [&](uint64_t target, const char* what, int w) {
    auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(120);
    while (sched.stats().bound < target) {
      if (std::chrono::steady_clock::now() > deadline) {
        std::fprintf(stderr, "%s %d timed out: bound %llu/%llu\n", what, w,
                     static_cast<unsigned long long>(sched.stats().bound), static_cast<unsigned long long>(target));
        return false;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    return true;
  };
  for (int w = 0; w < waves; ++w) {
    if (has_init) {
      if (sample_path) sampler::pause(true);
      Json init = Json::parse(slurp(dir + "/init.json"));
      std::vector<Json> ip(init.items().begin(), init.items().end());
      size_t in = ip.size();
      store->create_many("pods", std::move(ip));
      if (!wait_bound(bound + in, "init", w)) {
        sched.stop();
        return 1;
      }
      bound += in;
      if (sample_path) sampler::pause(false);
    }
    Json wave = Json::parse(slurp(dir + "/wave_" + std::to_string(w % 4) + ".json"));
    std::vector<Json> pgs(wave["podgroups"].items().begin(), wave["podgroups"].items().end());
    std::vector<Json> pods(wave["pods"].items().begin(), wave["pods"].items().end());
    size_t n = pods.size();
    // Workloads with pods that fit nowhere (Unschedulable) bind fewer.
    const size_t expect = static_cast<size_t>(wave["expect_bound"].as_int(static_cast<int64_t>(n)));
    auto t0 = std::chrono::steady_clock::now();
    // As bench.py (Wave.chunks_json): chunks of >= 64 pods ending on a gang
    // boundary, each chunk's PodGroups written just before its pods.
    {
      auto group_of = [](const Json& o) -> const std::string& {
        return o["metadata"]["labels"]["pod-group.scheduling.sigs.k8s.io"].as_string();
      };
      std::unordered_map<std::string, size_t> pg_at;
      for (size_t i = 0; i < pgs.size(); ++i) pg_at[pgs[i]["metadata"]["name"].as_string()] = i;
      std::vector<char> pg_done(pgs.size(), 0);
      std::vector<Json> chunk_pgs, chunk_pods;
      for (size_t i = 0; i < n; ++i) {
        const std::string g = group_of(pods[i]);
        if (auto it = pg_at.find(g); !g.empty() && it != pg_at.end() && !pg_done[it->second]) {
          pg_done[it->second] = 1;
          chunk_pgs.push_back(std::move(pgs[it->second]));
        }
        chunk_pods.push_back(std::move(pods[i]));
        const bool last = i + 1 == n;
        if (last || (chunk_pods.size() >= ObjectStore::kCreateChunk && (g.empty() || group_of(pods[i + 1]) != g))) {
          if (!chunk_pgs.empty()) store->create_many("podgroups", std::move(chunk_pgs));
          store->create_many("pods", std::move(chunk_pods));
          chunk_pgs.clear();
          chunk_pods.clear();
        }
      }
      std::vector<Json> rest;  // groups with no pod in this wave
      for (size_t i = 0; i < pgs.size(); ++i)
        if (!pg_done[i]) rest.push_back(std::move(pgs[i]));
      if (!rest.empty()) store->create_many("podgroups", std::move(rest));
    }
    auto t_created = std::chrono::steady_clock::now();
    if (!wait_bound(bound + expect, "wave", w)) {
      sched.stop();
      return 1;
    }
    auto t_bound = std::chrono::steady_clock::now();
    bound += expect;
    std::string ns = wave["namespace"].str_or("bench");
    store->delete_all("pods", has_init ? std::string() : ns);  // init pods may live in other namespaces
    store->delete_all("podgroups", ns);
    while (sched.cache().pod_count() > 0) std::this_thread::sleep_for(std::chrono::microseconds(100));
    auto t_end = std::chrono::steady_clock::now();
    double s = std::chrono::duration<double>(t_end - t0).count();
    auto ms = [](auto d) { return std::chrono::duration<double, std::milli>(d).count(); };
    total_s += s;
    total_pods += n;
    std::printf("wave %d: %zu pods in %.4fs (%.0f pods/s) create %.2fms to_bound %.2fms delete_drain %.2fms\n", w, n,
                s, n / s, ms(t_created - t0), ms(t_bound - t_created), ms(t_end - t_bound));
  }
  if (sample_path) sampler::dump(sample_path);
  sched.stop();
  std::printf("total: %zu pods in %.4fs (%.0f pods/s)\n", total_pods, total_s, total_pods / total_s);
  return 0;
}
