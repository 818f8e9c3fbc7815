#include "telemetry/amdsmi_sampler.h"

#include <dlfcn.h>

#include <cstdio>
#include <cstring>
#include <memory>

#include <amd_smi/amdsmi.h>

namespace xsched::telemetry {

namespace {

// Entry points resolved from libamd_smi at first use (types from the ROCm
// header the core is compiled against, so struct layouts match the library
// of the same image).
struct Api {
  decltype(&amdsmi_init) init = nullptr;
  decltype(&amdsmi_get_socket_handles) sockets = nullptr;
  decltype(&amdsmi_get_processor_handles) processors = nullptr;
  decltype(&amdsmi_get_processor_type) proc_type = nullptr;
  decltype(&amdsmi_get_gpu_bdf_id) bdf_id = nullptr;
  decltype(&amdsmi_get_gpu_activity) activity = nullptr;
  decltype(&amdsmi_get_gpu_vram_usage) vram = nullptr;
  decltype(&amdsmi_get_gpu_metrics_info) metrics = nullptr;
};
Api g_api;

template <typename F>
bool resolve(void* lib, const char* name, F& out) {
  out = reinterpret_cast<F>(dlsym(lib, name));
  return out != nullptr;
}

std::string format_bdf(uint64_t id) {
  char buf[32];
  std::snprintf(buf, sizeof buf, "%04x:%02x:%02x.%x", static_cast<unsigned>((id >> 32) & 0xffff),
                static_cast<unsigned>((id >> 8) & 0xff), static_cast<unsigned>((id >> 3) & 0x1f),
                static_cast<unsigned>(id & 0x7));
  return buf;
}

}  // namespace

AmdSmi& AmdSmi::get() {
  static AmdSmi* s = new AmdSmi();  // never destroyed: the library keeps global state
  return *s;
}

bool AmdSmi::init_locked() {
  tried_ = true;
  for (const char* path : {"libamd_smi.so", "/opt/rocm/lib/libamd_smi.so"}) {
    lib_ = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (lib_) break;
  }
  if (!lib_) {
    error_ = std::string("libamd_smi not loadable: ") + (dlerror() ? dlerror() : "?");
    return false;
  }
  Api& a = g_api;
  if (!resolve(lib_, "amdsmi_init", a.init) || !resolve(lib_, "amdsmi_get_socket_handles", a.sockets) ||
      !resolve(lib_, "amdsmi_get_processor_handles", a.processors) ||
      !resolve(lib_, "amdsmi_get_processor_type", a.proc_type) || !resolve(lib_, "amdsmi_get_gpu_bdf_id", a.bdf_id) ||
      !resolve(lib_, "amdsmi_get_gpu_activity", a.activity) || !resolve(lib_, "amdsmi_get_gpu_vram_usage", a.vram) ||
      !resolve(lib_, "amdsmi_get_gpu_metrics_info", a.metrics)) {
    error_ = "libamd_smi lacks an expected entry point";
    return false;
  }
  amdsmi_status_t st = a.init(AMDSMI_INIT_AMD_GPUS);
  if (st != AMDSMI_STATUS_SUCCESS) {
    error_ = "amdsmi_init failed (status " + std::to_string(static_cast<int>(st)) + ")";
    return false;
  }
  uint32_t nsock = 0;
  if (a.sockets(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS) {
    error_ = "amdsmi_get_socket_handles failed";
    return false;
  }
  std::vector<amdsmi_socket_handle> socks(nsock);
  if (nsock && a.sockets(&nsock, socks.data()) != AMDSMI_STATUS_SUCCESS) {
    error_ = "amdsmi_get_socket_handles failed";
    return false;
  }
  for (auto sh : socks) {
    uint32_t np = 0;
    if (a.processors(sh, &np, nullptr) != AMDSMI_STATUS_SUCCESS || np == 0) continue;
    std::vector<amdsmi_processor_handle> ph(np);
    if (a.processors(sh, &np, ph.data()) != AMDSMI_STATUS_SUCCESS) continue;
    for (auto h : ph) {
      processor_type_t t{};
      if (a.proc_type(h, &t) == AMDSMI_STATUS_SUCCESS && t == AMDSMI_PROCESSOR_TYPE_AMD_GPU) gpus_.push_back(h);
    }
  }
  if (gpus_.empty()) {
    error_ = "amd-smi found no AMD GPU";
    return false;
  }
  return true;
}

bool AmdSmi::available() {
  std::lock_guard<std::mutex> g(mu_);
  if (!tried_) ok_ = init_locked();
  return ok_;
}

std::vector<GpuSample> AmdSmi::sample() {
  std::lock_guard<std::mutex> g(mu_);
  if (!tried_) ok_ = init_locked();
  std::vector<GpuSample> out;
  if (!ok_) return out;
  const Api& a = g_api;
  for (size_t i = 0; i < gpus_.size(); ++i) {
    auto h = static_cast<amdsmi_processor_handle>(gpus_[i]);
    GpuSample s;
    s.index = static_cast<int>(i);
    uint64_t bdf = 0;
    if (a.bdf_id(h, &bdf) == AMDSMI_STATUS_SUCCESS) s.bdf = format_bdf(bdf);
    amdsmi_engine_usage_t u{};
    if (a.activity(h, &u) == AMDSMI_STATUS_SUCCESS) {
      s.gfx_activity = u.gfx_activity;
      s.umc_activity = u.umc_activity;
      s.mm_activity = u.mm_activity;
    }
    amdsmi_vram_usage_t v{};
    if (a.vram(h, &v) == AMDSMI_STATUS_SUCCESS) {
      s.vram_total_mb = v.vram_total;
      s.vram_used_mb = v.vram_used;
    }
    // The PMFW metrics table is large (~KBs); keep it off the stack.
    auto m = std::make_unique<amdsmi_gpu_metrics_t>();
    std::memset(m.get(), 0, sizeof(amdsmi_gpu_metrics_t));
    if (a.metrics(h, m.get()) == AMDSMI_STATUS_SUCCESS) {
      auto valid16 = [](uint16_t x) { return x != 0xffff; };
      if (valid16(m->current_socket_power) && m->current_socket_power) s.socket_power_w = m->current_socket_power;
      else if (valid16(m->average_socket_power)) s.socket_power_w = m->average_socket_power;
      if (valid16(m->temperature_hotspot)) s.temp_hotspot_c = m->temperature_hotspot;
      if (valid16(m->temperature_mem)) s.temp_mem_c = m->temperature_mem;
      if (s.gfx_activity < 0 && valid16(m->average_gfx_activity)) s.gfx_activity = m->average_gfx_activity;
      if (s.umc_activity < 0 && valid16(m->average_umc_activity)) s.umc_activity = m->average_umc_activity;
      for (int x = 0; x < AMDSMI_MAX_NUM_XCC; ++x) {
        uint32_t b = m->xcp_stats[0].gfx_busy_inst[x];
        if (b == UINT32_MAX) break;
        s.xcc_busy.push_back(b);
      }
      for (int l = 0; l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l) {
        s.xgmi_read_kb.push_back(m->xgmi_read_data_acc[l] == UINT64_MAX ? 0 : m->xgmi_read_data_acc[l]);
        s.xgmi_write_kb.push_back(m->xgmi_write_data_acc[l] == UINT64_MAX ? 0 : m->xgmi_write_data_acc[l]);
        uint16_t st = m->xgmi_link_status[l];
        s.xgmi_link_up.push_back(st == 0xffff ? -1 : (st ? 1 : 0));
      }
      if (valid16(m->xgmi_link_speed)) s.xgmi_link_speed = m->xgmi_link_speed;
      if (valid16(m->xgmi_link_width)) s.xgmi_link_width = m->xgmi_link_width;
      if (m->vram_max_bandwidth != UINT64_MAX) s.vram_max_bandwidth_gbs = static_cast<int64_t>(m->vram_max_bandwidth);
      s.firmware_timestamp_10ns = m->firmware_timestamp;
      if (valid16(m->num_partition)) s.num_partition = m->num_partition;
    }
    out.push_back(std::move(s));
  }
  return out;
}

}  // namespace xsched::telemetry
