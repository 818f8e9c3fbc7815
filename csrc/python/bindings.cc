// pybind11 bindings: the native core as the `_xsched` extension module.
//
// The Python control plane (flex_gpu_scheduler_amd/) drives the C++ store and
// scheduler through this module; hot paths (scheduling cycle, binding, watch
// fan-out) never enter Python. Bulk entry points take JSON text so a
// benchmark wave of thousands of pods crosses the boundary once.
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <map>
#include <set>

#include "api/types.h"
#include "common/alloc.h"
#include "common/json.h"
#include "common/quantity.h"
#include "rest/kube.h"
#include "scheduler/openloop.h"
#include "common/log.h"
#include "apiserver/apiserver.h"
#include "scheduler/scheduler.h"
#include "store/store.h"
#include "telemetry/amdsmi_sampler.h"
#include "tools/sampler.h"

namespace py = pybind11;
using namespace xsched;

namespace {

Json from_py(py::handle h) {
  if (h.is_none()) return Json();
  if (py::isinstance<py::bool_>(h)) return Json(h.cast<bool>());
  if (py::isinstance<py::int_>(h)) return Json(h.cast<int64_t>());
  if (py::isinstance<py::float_>(h)) return Json(h.cast<double>());
  if (py::isinstance<py::str>(h)) return Json(h.cast<std::string>());
  if (py::isinstance<py::dict>(h)) {
    Json o = Json::object();
    auto& m = o.members_mut();
    for (auto kv : h.cast<py::dict>()) m.emplace_back(py::str(kv.first).cast<std::string>(), from_py(kv.second));
    return o;
  }
  if (py::isinstance<py::list>(h) || py::isinstance<py::tuple>(h)) {
    Json a = Json::array();
    for (auto v : h) a.push_back(from_py(v));
    return a;
  }
  throw py::type_error("cannot convert object to JSON");
}

py::object to_py(const Json& j) {
  switch (j.type()) {
    case Json::Type::Null: return py::none();
    case Json::Type::Bool: return py::bool_(j.as_bool());
    case Json::Type::Int: return py::int_(j.as_int());
    case Json::Type::Double: return py::float_(j.as_double());
    case Json::Type::String: return py::str(j.as_string());
    case Json::Type::Array: {
      py::list l(j.size());
      size_t i = 0;
      for (const auto& v : j.items()) l[i++] = to_py(v);
      return std::move(l);
    }
    case Json::Type::Object: {
      py::dict d;
      for (const auto& kv : j.members()) d[py::str(kv.first)] = to_py(kv.second);
      return std::move(d);
    }
  }
  return py::none();
}

py::object ptr_to_py(const JsonPtr& p) { return p ? to_py(*p) : py::none(); }

Json json_arg(py::handle h) {
  if (py::isinstance<py::str>(h)) return Json::parse(h.cast<std::string>());
  return from_py(h);
}

// ApiClient implemented in Python (remote kube-apiserver / HTTP store).
class PyApiClient : public ApiClient {
 public:
  void bind(const Pod& pod, const std::string& node, const Json& annotations) override {
    py::gil_scoped_acquire g;
    py::function f = py::get_override(this, "bind");
    if (!f) throw std::runtime_error("PyApiClient.bind not implemented");
    f(pod.ns(), pod.name(), pod.uid(), node, to_py(annotations));
  }
  void delete_pod(const Pod& pod) override {
    py::gil_scoped_acquire g;
    py::function f = py::get_override(this, "delete_pod");
    if (!f) throw std::runtime_error("PyApiClient.delete_pod not implemented");
    f(pod.ns(), pod.name(), pod.uid());
  }
  void patch(const std::string& kind, const std::string& ns, const std::string& name, const Json& patch) override {
    py::gil_scoped_acquire g;
    py::function f = py::get_override(this, "patch");
    if (!f) throw std::runtime_error("PyApiClient.patch not implemented");
    f(kind, ns, name, to_py(patch));
  }
  void record_event(const std::string& kind, const std::string& ns, const std::string& name, const std::string& type,
                    const std::string& reason, const std::string& msg) override {
    py::gil_scoped_acquire g;
    py::function f = py::get_override(this, "record_event");
    if (f) f(kind, ns, name, type, reason, msg);
  }
};

py::dict pod_struct_summary(const Pod& pod);

py::dict pod_summary(const Json& obj) { return pod_struct_summary(*Pod::from_json(obj)); }

// The decoded fields of a Pod object (lister copies and parsed JSON compare
// equal field by field when the informer's bind fast path is exact).
py::dict pod_struct_summary(const Pod& pod) {
  const Pod* p = &pod;
  py::dict d;
  d["key"] = p->key();
  d["request"] = to_py(p->request().to_json());
  d["nonzero_request"] = to_py(p->nonzero_request().to_json());
  d["limits"] = to_py(p->limit_sum().to_json());
  const char* q[] = {"BestEffort", "Burstable", "Guaranteed"};
  d["qos"] = q[static_cast<int>(p->qos)];
  d["pod_group"] = p->pod_group;
  d["priority"] = p->priority;
  d["gpus"] = p->gpu.gpus;
  py::list parts;
  for (auto [g, pp] : p->gpu.partitions) parts.append(py::make_tuple(g, pp));
  d["partitions"] = parts;
  d["node_name"] = p->node_name;
  d["uid"] = p->uid();
  d["resource_version"] = p->meta.resource_version;
  d["labels"] = p->meta.labels.get();
  d["annotations"] = p->meta.annotations.get();
  d["phase"] = p->phase;
  d["scheduled_at"] = static_cast<int64_t>(p->scheduled_at);
  d["start_time"] = static_cast<int64_t>(p->start_time);
  d["template_hash"] = p->template_hash;
  d["spec_hash"] = p->spec_hash;
  d["scheduler_name"] = p->scheduler_name.str();
  d["host_ports"] = static_cast<int>(p->host_ports.size());
  return d;
}

py::dict node_info_dict(const NodeInfo& ni) {
  py::dict d;
  d["name"] = ni.name();
  d["pods"] = ni.num_pods();
  d["requested"] = to_py(ni.requested.to_json());
  d["allocatable"] = to_py(ni.allocatable.to_json());
  py::dict g;
  g["gpu_count"] = ni.gpu.gpu_count;
  g["mem_per_gpu"] = ni.gpu.mem_per_gpu;
  g["partitions"] = ni.gpu.parts;
  g["monopoly"] = ni.gpu.monopoly;
  py::list slots;
  for (int gi = 0; gi < ni.gpu.gpu_count; ++gi) {
    py::list ps;
    for (int s = ni.gpu.offset[gi]; s < ni.gpu.offset[gi + 1]; ++s) {
      const auto& sl = ni.gpu.slots[s];
      ps.append(py::make_tuple(sl.exclusive, sl.used_mem, sl.mem_pods));
    }
    slots.append(ps);
  }
  g["slots"] = slots;
  g["free_gpus"] = ni.gpu.free_gpus();
  g["free_xcds"] = ni.gpu.free_xcds();
  g["free_memory"] = ni.gpu.free_memory();
  d["gpu"] = g;
  return d;
}

// Python threads currently blocked inside a native wait with the GIL
// released. At interpreter exit the control plane stops every watcher and
// waits for this to reach zero: a daemon thread that re-acquires the GIL
// during finalization is terminated by CPython from inside pybind11's
// (noexcept) gil_scoped_release destructor, which aborts the process.
std::atomic<int> g_native_waiters{0};
struct WaiterGuard {
  WaiterGuard() { g_native_waiters.fetch_add(1); }
  ~WaiterGuard() { g_native_waiters.fetch_sub(1); }
};

void release_scheduler(Scheduler* s) {
  if (PyGILState_Check()) {
    py::gil_scoped_release r;
    delete s;
  } else {
    delete s;
  }
}

}  // namespace

PYBIND11_MODULE(_xsched, m) {
  m.doc() = "MI355X-native scheduler core (C++): object store, scheduling framework, plugins";
  tune_allocator();
  m.def("allocator_settings", [] { return tune_allocator(); },
        "The process allocator settings in effect (common/alloc.h).");

  py::register_exception<JsonError>(m, "JsonError");
  static py::exception<StoreError> store_exc(m, "StoreError");
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const StoreError& e) {
      py::object exc = py::handle(store_exc.ptr())(py::str(e.what()));
      exc.attr("code") = e.code();
      exc.attr("reason") = e.reason();
      PyErr_SetObject(store_exc.ptr(), exc.ptr());
    }
  });

  // ---- quantities / parsing helpers ----
  // Wall-clock sampling profiler of every thread (csrc/tools/sampler.h), for
  // stall diagnosis in Python-hosted runs (scripts/openloop_probe.py).
  m.def("sampler_start", [](int hz, size_t max_samples) { sampler::start(hz, max_samples); }, py::arg("hz") = 2000,
        py::arg("max_samples") = size_t{1} << 21);
  m.def("sampler_dump", [](const std::string& path) {
    py::gil_scoped_release nogil;
    sampler::dump(path);
  });
  m.def("parse_quantity", [](const std::string& s) {
    Quantity q = Quantity::parse(s);
    return py::make_tuple(q.milli_value(), q.value(), q.str());
  });
  m.def("canonical_quantity", [](const std::string& s) { return Quantity::parse(s).str(); });
  m.def("quantity_cmp", [](const std::string& a, const std::string& b) {
    return Quantity::parse(a).cmp(Quantity::parse(b));
  });
  // ResourceList arithmetic (k8s.io/apiserver/pkg/quota/v1 Add/Subtract/Max):
  // exact Quantity math; a sum keeps the format of the first non-zero operand.
  m.def("resource_list_op", [](const std::map<std::string, std::string>& a,
                               const std::map<std::string, std::string>& b, const std::string& op) {
    std::map<std::string, std::string> out;
    std::set<std::string> keys;
    for (const auto& kv : a) keys.insert(kv.first);
    for (const auto& kv : b) keys.insert(kv.first);
    for (const auto& k : keys) {
      auto ia = a.find(k), ib = b.find(k);
      bool ha = ia != a.end(), hb = ib != b.end();
      Quantity qa = ha ? Quantity::parse(ia->second) : Quantity();
      Quantity qb = hb ? Quantity::parse(ib->second) : Quantity();
      if (op == "max") {
        out[k] = (!ha || (hb && qb.cmp(qa) > 0) ? qb : qa).str();
        continue;
      }
      if (op != "add" && op != "sub") throw std::invalid_argument("op must be add, sub or max");
      if (qa.is_zero() && !ha) {
        qa = Quantity::from_int(0, qb.format());
      }
      if (op == "add") {
        qa.add(qb);
      } else {
        qa.sub(qb);
      }
      out[k] = qa.str();
    }
    return out;
  });
  m.def("pod_summary", [](py::handle obj) { return pod_summary(json_arg(obj)); });
  m.def("plugin_names", [] {
    register_builtin_plugins();
    return Registry::global().names();
  });
  m.def("json_roundtrip", [](const std::string& s) { return Json::parse(s).dump(); });
  // ---- live MI355X telemetry (libamd_smi) ----
  m.def("amdsmi_status", [] {
    auto& smi = telemetry::AmdSmi::get();
    py::gil_scoped_release nogil;
    bool ok = smi.available();
    py::gil_scoped_acquire gil;
    return py::make_tuple(ok, smi.error());
  });
  m.def("amdsmi_sample", [] {
    std::vector<telemetry::GpuSample> v;
    {
      py::gil_scoped_release nogil;
      v = telemetry::AmdSmi::get().sample();
    }
    py::list out;
    for (const auto& s : v) {
      py::dict d;
      d["index"] = s.index;
      d["bdf"] = s.bdf;
      d["gfx_activity"] = s.gfx_activity;
      d["umc_activity"] = s.umc_activity;
      d["mm_activity"] = s.mm_activity;
      d["xcc_busy"] = s.xcc_busy;
      d["vram_total_mb"] = s.vram_total_mb;
      d["vram_used_mb"] = s.vram_used_mb;
      d["socket_power_w"] = s.socket_power_w;
      d["temp_hotspot_c"] = s.temp_hotspot_c;
      d["temp_mem_c"] = s.temp_mem_c;
      d["xgmi_read_kb"] = s.xgmi_read_kb;
      d["xgmi_write_kb"] = s.xgmi_write_kb;
      d["xgmi_link_up"] = s.xgmi_link_up;
      d["xgmi_link_speed"] = s.xgmi_link_speed;
      d["xgmi_link_width"] = s.xgmi_link_width;
      d["vram_max_bandwidth_gbs"] = s.vram_max_bandwidth_gbs;
      d["firmware_timestamp_10ns"] = s.firmware_timestamp_10ns;
      d["num_partition"] = s.num_partition;
      out.append(std::move(d));
    }
    return out;
  });
  m.def("merge_patch", [](py::handle a, py::handle b) {
    Json x = json_arg(a);
    x.merge_patch(json_arg(b));
    return to_py(x);
  });
  // Two-way JSON merge patch from `a` to `b` (util.CreateMergePatch).
  m.def("diff_merge_patch",
        [](py::handle a, py::handle b) { return to_py(Json::diff_merge_patch(json_arg(a), json_arg(b))); });
  m.def("rfc3339", [](int64_t us) { return format_rfc3339(us); });
  m.def("native_waiters", [] { return g_native_waiters.load(); });
  m.def("parse_rfc3339", [](const std::string& s) { return parse_rfc3339(s); });
  // ---- native API server (apiserver/apiserver.h) ----
  py::class_<apiserver::Server, std::shared_ptr<apiserver::Server>>(m, "NativeApiServer")
      .def(py::init([](std::shared_ptr<ObjectStore> store, const std::string& host, int port, const std::string& token,
                       int bookmark_interval_ms, const std::string& tls_cert, const std::string& tls_key,
                       const std::string& client_ca) {
             apiserver::Options o;
             o.host = host;
             o.port = port;
             o.token = token;
             o.bookmark_interval_ms = bookmark_interval_ms;
             o.tls_cert_file = tls_cert;
             o.tls_key_file = tls_key;
             o.client_ca_file = client_ca;
             return std::make_shared<apiserver::Server>(std::move(store), o);
           }),
           py::arg("store"), py::arg("host") = "127.0.0.1", py::arg("port") = 0, py::arg("token") = "",
           py::arg("bookmark_interval_ms") = 10000, py::arg("tls_cert") = "", py::arg("tls_key") = "",
           py::arg("client_ca") = "")
      .def("start", &apiserver::Server::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &apiserver::Server::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &apiserver::Server::port)
      .def("requests", &apiserver::Server::requests)
      .def("connections", &apiserver::Server::connections);
  m.def("apply_json_patch", [](py::handle doc, py::handle ops) {
    return to_py(apiserver::apply_json_patch(json_arg(doc), json_arg(ops)));
  });

  // ---- native logging (common/log.h) ----
  m.def("set_log_verbosity", &xsched::log::set_verbosity, py::arg("v"));
  m.def("log_verbosity", &xsched::log::verbosity);
  m.def("set_log_json", &xsched::log::set_json, py::arg("json"));
  m.def("set_log_capture", &xsched::log::set_capture, py::arg("max_lines"));
  m.def("drain_log", &xsched::log::drain_captured);

  // ---- clock ----
  py::class_<FakeClock, std::shared_ptr<FakeClock>>(m, "FakeClock")
      .def(py::init<int64_t>(), py::arg("start_us") = 1'000'000'000)
      .def("now_us", &FakeClock::now_us)
      .def("advance", [](FakeClock& c, double seconds) { c.advance_us(static_cast<int64_t>(seconds * 1e6)); });

  // ---- store ----
  py::class_<Watcher, std::shared_ptr<Watcher>>(m, "Watcher")
      .def(
          "next",
          [](Watcher& w, int timeout_ms, size_t max) {
            std::vector<WatchEvent> evs;
            {
              WaiterGuard wg;
              py::gil_scoped_release r;
              evs = w.next(timeout_ms, max);
            }
            py::list out;
            for (const auto& e : evs)
              out.append(py::make_tuple(event_type_name(e.type), e.kind, ptr_to_py(e.obj), e.rv));
            return out;
          },
          py::arg("timeout_ms") = 0, py::arg("max") = 4096)
      .def(
          "next_json",
          [](Watcher& w, int timeout_ms, size_t max) {
            std::vector<WatchEvent> evs;
            {
              WaiterGuard wg;
              py::gil_scoped_release r;
              evs = w.next(timeout_ms, max);
            }
            py::list out;
            for (const auto& e : evs)
              out.append(py::make_tuple(event_type_name(e.type), e.kind, e.obj ? e.obj->dump() : std::string("null"), e.rv));
            return out;
          },
          py::arg("timeout_ms") = 0, py::arg("max") = 4096)
      .def("stop", &Watcher::stop)
      .def("pending", &Watcher::pending)
      .def_property_readonly("stopped", &Watcher::stopped);

  py::class_<ObjectStore, std::shared_ptr<ObjectStore>>(m, "Store")
      .def(py::init<>())
      .def("create",
           [](ObjectStore& s, const std::string& kind, py::handle obj) { return ptr_to_py(s.create(kind, json_arg(obj))); })
      .def("create_many",
           [](ObjectStore& s, const std::string& kind, py::handle objs) {
             // A JSON string is parsed element by element with the GIL
             // released and committed in PodGroup-aligned chunks, so the
             // informer and scheduler start on the first gangs while the rest
             // is still being parsed (see ObjectStore::create_chunked).
             if (py::isinstance<py::str>(objs)) {
               std::string text = objs.cast<std::string>();
               py::gil_scoped_release r;
               return s.create_chunked(kind, [&](const std::function<void(Json&&)>& emit) {
                 Json::parse_array_stream(text, emit);
               });
             }
             Json arr = json_arg(objs);
             std::vector<Json> v = std::move(arr.items_mut());
             py::gil_scoped_release r;
             return s.create_many(kind, std::move(v)).size();
           })
      .def("get",
           [](ObjectStore& s, const std::string& kind, const std::string& ns, const std::string& name) {
             return ptr_to_py(s.get(kind, ns, name));
           })
      .def("get_json",
           [](ObjectStore& s, const std::string& kind, const std::string& ns, const std::string& name) -> py::object {
             auto p = s.get(kind, ns, name);
             if (!p) return py::none();
             return py::str(p->dump());
           })
      .def(
          "list",
          [](ObjectStore& s, const std::string& kind, const std::string& ns) {
            int64_t rv = 0;
            auto items = s.list(kind, ns, &rv);
            py::list out;
            for (const auto& p : items) out.append(to_py(*p));
            return py::make_tuple(out, rv);
          },
          py::arg("kind"), py::arg("ns") = "")
      .def(
          "list_json",
          [](ObjectStore& s, const std::string& kind, const std::string& ns) {
            int64_t rv = 0;
            auto items = s.list(kind, ns, &rv);
            std::string out = "[";
            for (size_t i = 0; i < items.size(); ++i) {
              if (i) out += ",";
              items[i]->dump_to(out);
            }
            out += "]";
            return py::make_tuple(out, rv);
          },
          py::arg("kind"), py::arg("ns") = "")
      .def(
          "update",
          [](ObjectStore& s, const std::string& kind, py::handle obj, bool check_rv) {
            return ptr_to_py(s.update(kind, json_arg(obj), check_rv));
          },
          py::arg("kind"), py::arg("obj"), py::arg("check_rv") = true)
      .def("patch",
           [](ObjectStore& s, const std::string& kind, const std::string& ns, const std::string& name, py::handle p) {
             return ptr_to_py(s.patch(kind, ns, name, json_arg(p)));
           })
      .def(
          "delete",
          [](ObjectStore& s, const std::string& kind, const std::string& ns, const std::string& name, int64_t grace,
             const std::string& uid) { return ptr_to_py(s.remove(kind, ns, name, grace, uid)); },
          py::arg("kind"), py::arg("ns"), py::arg("name"), py::arg("grace_seconds") = 0, py::arg("uid") = "")
      .def("set_event_ttl_us", &ObjectStore::set_event_ttl_us, py::arg("ttl_us"))
      .def("delete_all", &ObjectStore::delete_all, py::arg("kind"), py::arg("ns") = "",
           py::call_guard<py::gil_scoped_release>())
      .def(
          "bind",
          [](ObjectStore& s, const std::string& ns, const std::string& name, const std::string& uid,
             const std::string& node, py::handle ann) { return ptr_to_py(s.bind(ns, name, uid, node, json_arg(ann))); },
          py::arg("ns"), py::arg("name"), py::arg("uid"), py::arg("node"), py::arg("annotations") = py::dict())
      .def(
          "watch",
          [](ObjectStore& s, std::vector<std::string> kinds, const std::string& ns, int64_t since) {
            return s.watch(std::set<std::string>(kinds.begin(), kinds.end()), ns, since);
          },
          py::arg("kinds") = std::vector<std::string>{}, py::arg("ns") = "", py::arg("since_rv") = 0)
      .def("unwatch", &ObjectStore::unwatch)
      .def_property_readonly("resource_version", &ObjectStore::resource_version)
      .def("count", &ObjectStore::count)
      .def(
          "add_fault",
          [](ObjectStore& s, const std::string& verb, const std::string& kind, double fail_prob, int delay_us,
             int remaining) { s.add_fault(FaultRule{verb, kind, fail_prob, delay_us, remaining}); },
          py::arg("verb"), py::arg("kind"), py::arg("fail_prob") = 0.0, py::arg("delay_us") = 0,
          py::arg("remaining") = -1)
      .def("clear_faults", &ObjectStore::clear_faults);

  // ---- API client trampoline ----
  py::class_<ApiClient, PyApiClient, std::shared_ptr<ApiClient>>(m, "ApiClient").def(py::init<>());

  // Native service mode (rest/kube.h): REST writes and the LIST/WATCH mirror.
  auto endpoint = [](const std::string& host, int port, const std::string& token, bool tls, const std::string& ca_file,
                     const std::string& ca_pem, const std::string& cert_file, const std::string& key_file,
                     const std::string& cert_pem, const std::string& key_pem, bool insecure, int timeout_ms,
                     double qps, int burst) {
    rest::Endpoint ep;
    ep.host = host;
    ep.port = port;
    ep.token = token;
    ep.timeout_ms = timeout_ms;
    ep.tls.enabled = tls;
    ep.tls.ca_file = ca_file;
    ep.tls.ca_pem = ca_pem;
    ep.tls.cert_file = cert_file;
    ep.tls.key_file = key_file;
    ep.tls.cert_pem = cert_pem;
    ep.tls.key_pem = key_pem;
    ep.tls.insecure = insecure;
    ep.qps = qps;
    ep.burst = burst;
    return ep;
  };
  py::class_<rest::Endpoint>(m, "RestEndpoint")
      .def(py::init(endpoint), py::arg("host"), py::arg("port"), py::arg("token") = "", py::arg("tls") = false,
           py::arg("ca_file") = "", py::arg("ca_pem") = "", py::arg("cert_file") = "", py::arg("key_file") = "",
           py::arg("cert_pem") = "", py::arg("key_pem") = "", py::arg("insecure") = false,
           py::arg("timeout_ms") = 30000, py::arg("qps") = 0.0, py::arg("burst") = 0);
  py::class_<rest::RestApiClient, ApiClient, std::shared_ptr<rest::RestApiClient>>(m, "RestApiClient")
      .def(py::init<rest::Endpoint>())
      .def("requests", &rest::RestApiClient::requests)
      .def(
          "bind_json",
          [](rest::RestApiClient& c, py::handle pod, const std::string& node, py::handle ann) {
            auto p = Pod::from_json(json_arg(pod));
            Json a = json_arg(ann);
            py::gil_scoped_release r;
            c.bind(*p, node, a);
          },
          py::arg("pod"), py::arg("node"), py::arg("annotations") = py::dict());
  py::class_<rest::RemoteMirror, std::shared_ptr<rest::RemoteMirror>>(m, "RemoteMirror")
      .def(py::init<rest::Endpoint, std::shared_ptr<ObjectStore>, std::vector<std::string>>())
      .def("start", &rest::RemoteMirror::start)
      .def("wait_synced", &rest::RemoteMirror::wait_synced, py::call_guard<py::gil_scoped_release>())
      .def("stop", &rest::RemoteMirror::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("applied", &rest::RemoteMirror::applied)
      .def_property_readonly("relists", &rest::RemoteMirror::relists)
      .def("last_error", &rest::RemoteMirror::last_error);

  // ---- scheduler ----
  // Open-loop gang arrivals (scheduler/openloop.h): gangs_json = [{"podgroup":
  // {...}, "pods": [...]}, ...]; returns per-gang timelines in microseconds.
  m.def(
      "run_open_loop",
      [](ObjectStore& store, Scheduler& sched, const std::string& gangs_json, std::vector<int64_t> offsets_us,
         int64_t hold_us, int64_t timeout_us) {
        std::vector<OpenLoopGang> gangs;
        {
          Json arr = Json::parse(gangs_json);
          gangs.reserve(arr.size());
          for (const auto& g : arr.items()) {
            OpenLoopGang og;
            og.pod_group = g["podgroup"];
            og.pods.assign(g["pods"].items().begin(), g["pods"].items().end());
            gangs.push_back(std::move(og));
          }
        }
        OpenLoopResult r;
        {
          py::gil_scoped_release rel;
          r = run_open_loop(store, sched, std::move(gangs), offsets_us, hold_us, timeout_us);
        }
        py::list out;
        for (const auto& g : r.gangs) {
          py::dict d;
          d["size"] = g.size;
          d["create_us"] = g.create_us;
          d["first_enqueue_us"] = g.first_enqueue_us;
          d["admit_us"] = g.admit_us;
          d["bound_us"] = g.bound_us;
          d["nodes"] = g.nodes;
          d["hostable"] = g.hostable;
          out.append(d);
        }
        py::dict res;
        res["gangs"] = out;
        res["wall_us"] = r.wall_us;
        res["late_us"] = r.late_us;
        res["delete_late_us"] = r.delete_late_us;
        res["max_in_flight_pods"] = r.max_in_flight_pods;
        res["max_held_pods"] = r.max_held_pods;
        res["timeline"] = r.timeline;
        return res;
      },
      py::arg("store"), py::arg("sched"), py::arg("gangs_json"), py::arg("offsets_us"), py::arg("hold_us"),
      py::arg("timeout_us") = 10'000'000);

  py::class_<Scheduler, std::shared_ptr<Scheduler>>(m, "Scheduler")
      .def(py::init([](std::shared_ptr<ObjectStore> store, py::handle config, std::shared_ptr<FakeClock> clock,
                       std::shared_ptr<ApiClient> client) {
             Json cfg = json_arg(config);
             std::shared_ptr<Clock> c = clock;
             Scheduler* s;
             {
               py::gil_scoped_release r;
               s = new Scheduler(store, cfg, c, client);
             }
             return std::shared_ptr<Scheduler>(s, release_scheduler);
           }),
           py::arg("store"), py::arg("config"), py::arg("clock") = nullptr, py::arg("client") = nullptr)
      .def("start", &Scheduler::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &Scheduler::stop, py::call_guard<py::gil_scoped_release>())
      .def("sync_informers", &Scheduler::sync_informers, py::arg("timeout_ms") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("schedule_one", &Scheduler::schedule_one, py::arg("timeout_ms") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("wait_idle", &Scheduler::wait_idle, py::arg("timeout_ms") = 10000, py::call_guard<py::gil_scoped_release>())
      .def("stats",
           [](Scheduler& s) {
             auto st = s.stats();
             py::dict d;
             d["attempts"] = st.attempts;
             d["scheduled"] = st.scheduled;
             d["unschedulable"] = st.unschedulable;
             d["errors"] = st.errors;
             d["bound"] = st.bound;
             d["bind_failures"] = st.bind_failures;
             d["preemption_attempts"] = st.preemption_attempts;
             d["eq_filter_hits"] = st.eq_filter_hits;
             d["eq_filter_misses"] = st.eq_filter_misses;
             d["scan_memo_served"] = st.scan_memo_served;
             d["scan_memo_mismatches"] = st.scan_memo_mismatches;
             d["inflight_bindings"] = s.inflight_bindings();
             d["bind_threads"] = s.bind_threads();
             return d;
           })
      .def(
          "gang_records",
          [](Scheduler& s, bool clear) {
            py::list out;
            for (const auto& r : s.gang_records(clear)) {
              py::dict d;
              d["pod_group"] = r.pg;
              d["size"] = r.size;
              d["first_enqueue_us"] = r.first_enqueue_us;
              d["admit_us"] = r.admit_us;
              d["bound_us"] = r.bound_us;
              d["nodes"] = static_cast<int>(r.nodes.size());
              d["hostable"] = r.hostable;
              out.append(d);
            }
            return out;
          },
          py::arg("clear") = false)
      .def(
          "gang_denials",
          [](Scheduler& s, bool clear) {
            uint64_t total = 0;
            auto v = s.gang_denials(clear, &total);
            py::list out;
            for (const auto& d : v) {
              py::dict e;
              e["pod_group"] = d.pg;
              e["why"] = d.why;
              e["cause"] = d.cause;
              e["t_us"] = d.t_us;
              e["min_member"] = d.min_member;
              e["assigned"] = d.assigned;
              e["need_gpus"] = d.need_gpus;
              e["cache_free"] = d.cache_free;
              e["cache_max_node_free"] = d.cache_max_node_free;
              e["assumed_held"] = d.assumed_held;
              e["store_free"] = d.store_free;
              e["store_max_node_free"] = d.store_max_node_free;
              e["waiting_at_permit"] = d.waiting_at_permit;
              e["in_binding"] = d.in_binding;
              out.append(e);
            }
            return py::make_tuple(total, out);
          },
          py::arg("clear") = false)
      .def("gang_parks", [](Scheduler& s, bool clear) { return s.gang_parks(clear); }, py::arg("clear") = false)
      .def("queue_counts",
           [](Scheduler& s) {
             auto c = s.queue().counts();
             py::dict d;
             d["active"] = c.active;
             d["backoff"] = c.backoff;
             d["unschedulable"] = c.unschedulable;
             d["parked"] = c.parked;
             d["in_flight"] = s.queue().in_flight();
             d["activation_marks"] = s.queue().pending_activations();
             return d;
           })
      // NextPod without a scheduling cycle (the reference's integration tests
      // pop the queue of a scheduler that is not running, qos_test.go:129).
      .def(
          "next_pod",
          [](Scheduler& s, int timeout_ms) -> py::object {
            QueuedPodInfoPtr q;
            {
              py::gil_scoped_release r;
              q = s.queue().pop(timeout_ms);
            }
            if (!q) return py::none();
            return py::str(q->pod->key());
          },
          py::arg("timeout_ms") = 0)
      .def("flush_backoff", [](Scheduler& s) { s.queue().flush_backoff_completed(); })
      .def("flush_unschedulable", [](Scheduler& s) { s.queue().flush_unschedulable_leftover(); })
      .def("move_all", [](Scheduler& s) { s.queue().move_all_to_active_or_backoff(ClusterEvent{"*", kAll, ""}); })
      .def("poke_timers", &Scheduler::sync_informers, py::arg("timeout_ms") = 0)
      .def("run_timers", [](Scheduler& s) {
        py::gil_scoped_release r;
        s.timers().poke_and_drain();
      })
      .def("node_info",
           [](Scheduler& s, const std::string& name) -> py::object {
             auto ni = s.cache().node_info_copy(name);
             if (!ni) return py::none();
             return node_info_dict(*ni);
           })
      .def("node_names", [](Scheduler& s) { return s.cache().node_names(); })
      .def("wait_bound",
           [](Scheduler& s, uint64_t target, double timeout_s) {
             py::gil_scoped_release r;
             return s.wait_bound(target, static_cast<int64_t>(timeout_s * 1e6));
           })
      .def("wait_cache_empty",
           [](Scheduler& s, double timeout_s) {
             py::gil_scoped_release r;
             return s.wait_cache_empty(static_cast<int64_t>(timeout_s * 1e6));
           })
      .def("cache_counts",
           [](Scheduler& s) {
             py::dict d;
             d["nodes"] = s.cache().node_count();
             d["pods"] = s.cache().pod_count();
             d["assumed"] = s.cache().assumed_count();
             return d;
           })
      .def("lister_pod",
           [](Scheduler& s, const std::string& ns, const std::string& name) -> py::object {
             auto p = s.informers().pod(ns, name);
             if (!p) return py::none();
             return pod_struct_summary(*p);
           })
      .def("lister_counts",
           [](Scheduler& s) {
             py::dict d;
             d["pods"] = s.informers().pod_count();
             d["podgroups"] = s.informers().pod_groups().size();
             d["elasticquotas"] = s.informers().elastic_quotas().size();
             return d;
           })
      .def("assigned_in_group", [](Scheduler& s, const std::string& pg) { return s.cache().assigned_in_group(pg); })
      .def("waiting_pods",
           [](Scheduler& s) {
             py::list out;
             for (const auto& fw : s.frameworks())
               fw->handle().waiting_pods->iterate([&](const WaitingPodPtr& wp) {
                 out.append(py::make_tuple(wp->pod()->key(), wp->node(), wp->pending_plugins()));
               });
             return out;
           })
      .def("explain",
           [](Scheduler& s, py::handle pod) {
             Json j = json_arg(pod);
             Json out;
             {
               py::gil_scoped_release r;
               out = s.explain(j);
             }
             return to_py(out);
           })
      .def("check_cache",
           [](Scheduler& s) {
             Json out;
             {
               py::gil_scoped_release r;
               out = s.check_cache();
             }
             return to_py(out);
           })
      .def("dump_cache",
           [](Scheduler& s) {
             Json out;
             {
               py::gil_scoped_release r;
               out = s.dump_cache();
             }
             return to_py(out);
           })
      .def("score_benchmark",
           [](Scheduler& s, py::handle pod, int iterations) {
             Json j = json_arg(pod);
             Json out;
             {
               py::gil_scoped_release r;
               s.score_benchmark(j, iterations, &out);
             }
             return to_py(out);
           },
           py::arg("pod"), py::arg("iterations") = 100)
      .def("metrics_text", [](Scheduler& s) { return s.metrics().expose(); })
      .def("loop_age_seconds", &Scheduler::loop_age_seconds)
      .def(
          "plugin_call",
          [](Scheduler& s, const std::string& plugin, const std::string& point, py::handle args) {
            Json a = json_arg(args);
            Json out;
            {
              py::gil_scoped_release r;
              out = s.plugin_call(plugin, point, a);
            }
            return to_py(out);
          },
          py::arg("plugin"), py::arg("point"), py::arg("args"))
      .def("set_trace",
           [](Scheduler& s, bool on, size_t capacity) {
             if (capacity) s.tracer().set_capacity(capacity);
             s.tracer().enable(on);
           },
           py::arg("on"), py::arg("capacity") = 0)
      .def("trace_json", [](Scheduler& s) { return s.tracer().chrome_json(); })
      .def("clear_trace", [](Scheduler& s) { s.tracer().clear(); })
      .def("profiles", [](Scheduler& s) {
        py::list out;
        for (const auto& fw : s.frameworks()) {
          py::dict d;
          d["schedulerName"] = fw->profile_name();
          py::dict pts;
          for (const auto& [pt, names] : fw->config().enabled) pts[ext_point_name(pt)] = names;
          d["plugins"] = pts;
          out.append(d);
        }
        return out;
      });
}
