// mi355x-rocr-devsetup: where do the ~10 ms of per-device set-up after
// hsa_init go? (measurement tool, not shipped)
//
// Runs every ROCr call the container entrypoint makes between hsa_init and the
// verified MFMA tile one at a time, on the first GPU agent, timing each and
// sampling what the threads are blocked in meanwhile (init_sampler.h; ioctls
// carry their command byte: kfd 0x02 CREATE_QUEUE, 0x16 ALLOC_MEMORY_OF_GPU,
// 0x18 MAP_MEMORY_TO_GPU, ...).
//
//   mi355x-rocr-devsetup HSACO [--order queue-first|alloc-first|code-first] -> one JSON line
#include <dirent.h>
#include <dlfcn.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <time.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <iterator>
#include <string>
#include <vector>

#include "../src/health/init_sampler.h"
#include "../src/health/liveness_kernel.h"
#ifdef MI355X_IOCTL_TRACE
#include "ioctl_trace.h"  // build with -DMI355X_IOCTL_TRACE -rdynamic: per-step ioctl wall times
#endif

namespace {

double now_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

#define FN(name) decltype(&::name) name = reinterpret_cast<decltype(&::name)>(dlsym(lib, #name))

struct Step {
  std::string name;
  double ms = 0;
  hsa_status_t status = HSA_STATUS_SUCCESS;
  std::string profile;
  std::string queues;
  std::string ioctls = "null";
};

// This process' kfd queues (/sys/class/kfd/kfd/proc/<pid>/queues/<qid>/type):
// the queues ROCr created behind the API, e.g. {"ComputeAQL":2,"SDMA":1}.
std::string kfd_queues() {
  char dir[96];
  std::snprintf(dir, sizeof(dir), "/sys/class/kfd/kfd/proc/%d/queues", static_cast<int>(getpid()));
  DIR* d = opendir(dir);
  if (!d) return "null";
  std::vector<std::pair<std::string, int>> counts;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    std::string p = std::string(dir) + "/" + e->d_name + "/type";
    std::ifstream f(p);
    std::string t;
    std::getline(f, t);
    if (t.empty()) t = "?";
    bool found = false;
    for (auto& kv : counts)
      if (kv.first == t) ++kv.second, found = true;
    if (!found) counts.emplace_back(t, 1);
  }
  closedir(d);
  std::string o = "{";
  for (size_t i = 0; i < counts.size(); ++i)
    o += (i ? ",\"" : "\"") + counts[i].first + "\":" + std::to_string(counts[i].second);
  return o + "}";
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s HSACO [--order queue-first|alloc-first|code-first]\n", argv[0]);
    return 2;
  }
  std::string order = "queue-first";
  for (int i = 2; i + 1 < argc; ++i)
    if (std::strcmp(argv[i], "--order") == 0) order = argv[i + 1];
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<char> co((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (co.empty()) {
    std::printf("{\"ok\":false,\"error\":\"cannot read %s\"}\n", argv[1]);
    return 2;
  }
  void* lib = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!lib) lib = dlopen("/opt/rocm/lib/libhsa-runtime64.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!lib) {
    std::printf("{\"ok\":false,\"error\":\"dlopen: %s\"}\n", dlerror());
    return 2;
  }
  FN(hsa_init);
  FN(hsa_iterate_agents);
  FN(hsa_agent_get_info);
  FN(hsa_amd_agent_iterate_memory_pools);
  FN(hsa_amd_memory_pool_get_info);
  FN(hsa_amd_memory_pool_allocate);
  FN(hsa_amd_agents_allow_access);
  FN(hsa_queue_create);
  FN(hsa_signal_create);
  FN(hsa_signal_store_screlease);
  FN(hsa_amd_pointer_info);
  FN(hsa_signal_wait_scacquire);
  FN(hsa_queue_add_write_index_screlease);
  FN(hsa_code_object_reader_create_from_memory);
  FN(hsa_executable_create_alt);
  FN(hsa_executable_load_agent_code_object);
  FN(hsa_executable_freeze);
  FN(hsa_executable_get_symbol_by_name);
  FN(hsa_executable_symbol_get_info);
  FN(hsa_amd_profiling_set_profiler_enabled);

#ifdef MI355X_IOCTL_TRACE
  const size_t io_init = ioctl_trace_mark();
#endif
  const double t0 = now_ms();
  hsa_status_t s = hsa_init();
  const double t_init = now_ms() - t0;
#ifdef MI355X_IOCTL_TRACE
  const std::string init_ioctls = ioctl_trace_json(io_init);
#else
  const std::string init_ioctls = "null";
#endif
  if (s != HSA_STATUS_SUCCESS) {
    std::printf("{\"ok\":false,\"error\":\"hsa_init %d\"}\n", static_cast<int>(s));
    return 1;
  }
  struct Ctx {
    hsa_agent_t gpu{}, cpu{};
    hsa_amd_memory_pool_t coarse{}, fine{}, kernarg{};
    bool has_gpu = false, has_cpu = false;
    bool gpu_pass = false;  // coarse (HBM) pool from the GPU agent only: the CPU agent has a coarse system pool too
    decltype(&::hsa_agent_get_info) get_info;
    decltype(&::hsa_amd_memory_pool_get_info) pool_info;
  } c;
  c.get_info = hsa_agent_get_info;
  c.pool_info = hsa_amd_memory_pool_get_info;
  hsa_iterate_agents(
      [](hsa_agent_t a, void* p) {
        auto* c = static_cast<Ctx*>(p);
        hsa_device_type_t t;
        c->get_info(a, HSA_AGENT_INFO_DEVICE, &t);
        if (t == HSA_DEVICE_TYPE_GPU && !c->has_gpu) c->gpu = a, c->has_gpu = true;
        if (t == HSA_DEVICE_TYPE_CPU && !c->has_cpu) c->cpu = a, c->has_cpu = true;
        return HSA_STATUS_SUCCESS;
      },
      &c);
  if (!c.has_gpu || !c.has_cpu) {
    std::printf("{\"ok\":false,\"error\":\"no gpu/cpu agent\"}\n");
    return 1;
  }
  auto pick = [](hsa_amd_memory_pool_t p, void* d) {
    auto* c = static_cast<Ctx*>(d);
    hsa_amd_segment_t seg;
    c->pool_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t fl = 0;
    c->pool_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
    if (!c->gpu_pass) {
      if (fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) c->kernarg = p;
      else if ((fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !c->fine.handle) c->fine = p;
    } else if ((fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && !c->coarse.handle) {
      bool alloc_ok = false;
      c->pool_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc_ok);
      if (alloc_ok) c->coarse = p;
    }
    return HSA_STATUS_SUCCESS;
  };
  hsa_amd_agent_iterate_memory_pools(c.cpu, pick, &c);
  c.gpu_pass = true;
  hsa_amd_agent_iterate_memory_pools(c.gpu, pick, &c);
  if (!c.kernarg.handle || !c.fine.handle || !c.coarse.handle) {
    std::printf("{\"ok\":false,\"error\":\"missing pool (kernarg %d fine %d coarse %d)\"}\n", c.kernarg.handle != 0,
                c.fine.handle != 0, c.coarse.handle != 0);
    return 1;
  }

  hsa_queue_t *q1 = nullptr, *q2 = nullptr;
  hsa_signal_t sig{};
  float* out = nullptr;
  uint32_t* meta = nullptr;
  float* scratch = nullptr;
  mi355x_liveness_args* kargs = nullptr;
  hsa_code_object_reader_t rd{};
  hsa_executable_t exe{};
  uint64_t kobj = 0;
  uint32_t pseg = 0, gseg = 0;

  std::vector<std::pair<std::string, std::function<hsa_status_t()>>> queue_steps = {
      {"queue_create", [&] { return hsa_queue_create(c.gpu, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX,
                                                      UINT32_MAX, &q1); }},
      {"profiler_enable", [&] { return hsa_amd_profiling_set_profiler_enabled(q1, 1); }},
      {"queue_create_2nd", [&] { return hsa_queue_create(c.gpu, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr,
                                                          UINT32_MAX, UINT32_MAX, &q2); }},
      {"signal_create", [&] { return hsa_signal_create(1, 0, nullptr, &sig); }},
  };
  std::vector<std::pair<std::string, std::function<hsa_status_t()>>> alloc_steps = {
      {"alloc_fine_4k", [&] { return hsa_amd_memory_pool_allocate(c.fine, 4096, 0, reinterpret_cast<void**>(&out)); }},
      {"allow_fine_4k", [&] { return hsa_amd_agents_allow_access(1, &c.gpu, nullptr, out); }},
      {"alloc_fine_64", [&] { return hsa_amd_memory_pool_allocate(c.fine, 64, 0, reinterpret_cast<void**>(&meta)); }},
      {"allow_fine_64", [&] { return hsa_amd_agents_allow_access(1, &c.gpu, nullptr, meta); }},
      {"alloc_kernarg", [&] { return hsa_amd_memory_pool_allocate(c.kernarg, 256, 0, reinterpret_cast<void**>(&kargs)); }},
      {"allow_kernarg", [&] { return hsa_amd_agents_allow_access(1, &c.gpu, nullptr, kargs); }},
      {"alloc_coarse_4k", [&] { return hsa_amd_memory_pool_allocate(c.coarse, MI355X_SCRATCH_FLOATS * sizeof(float), 0,
                                                                     reinterpret_cast<void**>(&scratch)); }},
  };
  std::vector<std::pair<std::string, std::function<hsa_status_t()>>> code_steps = {
      {"co_reader", [&] { return hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rd); }},
      {"exe_create", [&] { return hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT,
                                                             nullptr, &exe); }},
      {"co_load", [&] { return hsa_executable_load_agent_code_object(exe, c.gpu, rd, nullptr, nullptr); }},
      {"exe_freeze", [&] { return hsa_executable_freeze(exe, nullptr); }},
      {"symbol", [&] {
         hsa_executable_symbol_t sym{};
         hsa_status_t st = hsa_executable_get_symbol_by_name(exe, "mi355x_mfma_liveness.kd", &c.gpu, &sym);
         if (st != HSA_STATUS_SUCCESS) return st;
         hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &kobj);
         hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &pseg);
         hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &gseg);
         return HSA_STATUS_SUCCESS;
       }},
  };
  auto dispatch = [&]() -> hsa_status_t {
    if (!out || !meta || !kargs || !scratch || !kobj || !q1) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
    // the kernel writes scratch from the GPU: it must be this GPU's own memory
    hsa_amd_pointer_info_t pi{};
    pi.size = sizeof(pi);
    if (hsa_amd_pointer_info(scratch, &pi, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        pi.agentOwner.handle != c.gpu.handle || pi.type != HSA_EXT_POINTER_TYPE_HSA)
      return HSA_STATUS_ERROR_INVALID_ARGUMENT;
    hsa_signal_store_screlease(sig, 1);
    std::memset(out, 0xFF, 4096);
    std::memset(meta, 0, 64);
    std::memset(kargs, 0, 256);
    kargs->out = out;
    kargs->meta = meta;
    kargs->scratch = scratch;
    kargs->nonce = 7;
    kargs->iters = 1;
    const uint64_t idx = hsa_queue_add_write_index_screlease(q1, 1);
    auto* pkt = static_cast<hsa_kernel_dispatch_packet_t*>(q1->base_address) + (idx & (q1->size - 1));
    std::memset(reinterpret_cast<char*>(pkt) + 4, 0, sizeof(*pkt) - 4);
    pkt->workgroup_size_x = 64;
    pkt->workgroup_size_y = pkt->workgroup_size_z = 1;
    pkt->grid_size_x = 64;
    pkt->grid_size_y = pkt->grid_size_z = 1;
    pkt->private_segment_size = pseg;
    pkt->group_segment_size = gseg;
    pkt->kernel_object = kobj;
    pkt->kernarg_address = kargs;
    pkt->completion_signal = sig;
    const uint16_t header = static_cast<uint16_t>(
        (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
        (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
        (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
    __atomic_store_n(reinterpret_cast<uint32_t*>(pkt),
                     header | (static_cast<uint32_t>(1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS) << 16),
                     __ATOMIC_RELEASE);
    hsa_signal_store_screlease(q1->doorbell_signal, static_cast<hsa_signal_value_t>(idx));
    const double dl = now_ms() + 5000;
    while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, 20 * 1000 * 1000ull, HSA_WAIT_STATE_BLOCKED) >= 1)
      if (now_ms() > dl) return HSA_STATUS_ERROR;
    return meta[MI355X_META_MAGIC] == MI355X_PROBE_MAGIC ? HSA_STATUS_SUCCESS : HSA_STATUS_ERROR;
  };

  std::vector<std::pair<std::string, std::function<hsa_status_t()>>> plan;
  auto add = [&](auto& v) { plan.insert(plan.end(), v.begin(), v.end()); };
  if (order == "alloc-first") { add(alloc_steps); add(queue_steps); add(code_steps); }
  else if (order == "code-first") { add(code_steps); add(queue_steps); add(alloc_steps); }
  else { add(queue_steps); add(alloc_steps); add(code_steps); }
  plan.emplace_back("dispatch_wait", dispatch);
  plan.emplace_back("dispatch_wait_2nd", dispatch);

  std::vector<Step> steps;
  bool ok = true;
  const double t_dev0 = now_ms();
  for (auto& [name, fn] : plan) {
    mi355x::InitSampler smp(100);
    smp.start();
#ifdef MI355X_IOCTL_TRACE
    const size_t io0 = ioctl_trace_mark();
#endif
    const double a = now_ms();
    const hsa_status_t st = fn();
    const double b = now_ms();
    smp.stop();
    steps.push_back({name, b - a, st, smp.json(), kfd_queues()});
#ifdef MI355X_IOCTL_TRACE
    steps.back().ioctls = ioctl_trace_json(io0);
#endif
    if (st != HSA_STATUS_SUCCESS) {
      ok = false;
      break;
    }
  }
  const double t_dev = now_ms() - t_dev0;
  std::string o = "{\"ok\":" + std::string(ok ? "true" : "false") + ",\"order\":\"" + order +
                  "\",\"hsa_init_ms\":" + std::to_string(t_init) + ",\"hsa_init_ioctls\":" + init_ioctls + ",\"device_setup_ms\":" + std::to_string(t_dev) +
                  ",\"steps\":[";
  for (size_t i = 0; i < steps.size(); ++i) {
    if (i) o += ",";
    o += "{\"name\":\"" + steps[i].name + "\",\"ms\":" + std::to_string(steps[i].ms) +
         ",\"status\":" + std::to_string(static_cast<int>(steps[i].status)) + ",\"profile\":" + steps[i].profile +
         ",\"kfd_queues\":" + steps[i].queues + ",\"ioctls\":" + steps[i].ioctls + "}";
  }
  o += "]}";
  std::printf("%s\n", o.c_str());
  std::fflush(stdout);
  std::_Exit(ok ? 0 : 1);  // teardown is not what this tool measures
}
