// mi355x-rocr-queue-origin: which ROCr call creates which kfd queue, and what
// each one costs in host memory (measurement tool, not shipped).
//
// The persistent probe server holds two 181 MB context-save (CWSR) areas per
// GPU (profiles/archive/measurements_r1_r3.md §3f, §3i): its own queue and one ROCr creates
// behind the API. This tool interposes ioctl() (the executable exports it,
// -rdynamic; ROCr's thunk resolves ioctl against the executable first) and,
// for every AMDKFD_IOC_CREATE_QUEUE, records the arguments the thunk passes
// (queue type, ring size, CWSR size, control-stack size, priority) and the
// call stack (module + offset, nearest exported symbol); for every
// AMDKFD_IOC_SVM the registered range size. It then runs the steps a probe
// server runs, one at a time, with RSS and the process' kfd queues after
// each:
//
//   hsa_init -> hsa_queue_create (the probe queue) -> code object load +
//   freeze -> a signal + a kernarg allocation -> a second hsa_queue_create
//
//   g++ -O1 -g -std=c++17 -rdynamic -I/opt/rocm/include native/tools/rocr_queue_origin.cpp -o rqo -ldl -pthread
//   ROCR_VISIBLE_DEVICES=0 ./rqo <code object> [--code-first]   -> one JSON line
#include <dirent.h>
#include <dlfcn.h>
#include <execinfo.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <linux/kfd_ioctl.h>
#include <stdarg.h>
#include <sys/ioctl.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <mutex>
#include <string>
#include <vector>

namespace {

struct QueueCall {
  unsigned queue_type, ring_size, priority, percentage, cwsr_size, ctl_stack_size;
  unsigned long long eop_size;
  int rc;
  std::vector<std::string> stack;
};

std::mutex g_mu;
std::vector<QueueCall> g_queues;
std::vector<unsigned long long> g_svm_sizes;
int g_ioctls = 0;

std::string frame(void* pc) {
  Dl_info info{};
  char buf[256];
  if (dladdr(pc, &info) && info.dli_fname) {
    const char* lib = std::strrchr(info.dli_fname, '/');
    lib = lib ? lib + 1 : info.dli_fname;
    const unsigned long off = reinterpret_cast<unsigned long>(pc) - reinterpret_cast<unsigned long>(info.dli_fbase);
    if (info.dli_sname)
      std::snprintf(buf, sizeof(buf), "%s+0x%lx (%s+0x%lx)", lib, off, info.dli_sname,
                    reinterpret_cast<unsigned long>(pc) - reinterpret_cast<unsigned long>(info.dli_saddr));
    else
      std::snprintf(buf, sizeof(buf), "%s+0x%lx", lib, off);
    return buf;
  }
  std::snprintf(buf, sizeof(buf), "%p", pc);
  return buf;
}

}  // namespace

extern "C" int ioctl(int fd, unsigned long request, ...) {
  using fn_t = int (*)(int, unsigned long, ...);
  static fn_t real = reinterpret_cast<fn_t>(dlsym(RTLD_NEXT, "ioctl"));
  va_list ap;
  va_start(ap, request);
  void* arg = va_arg(ap, void*);
  va_end(ap);
  const int r = real(fd, request, arg);
  if (_IOC_TYPE(request) == 'K') {
    std::lock_guard<std::mutex> lk(g_mu);
    ++g_ioctls;
    if (_IOC_NR(request) == 0x02) {
      const auto* a = static_cast<const kfd_ioctl_create_queue_args*>(arg);
      QueueCall q{a->queue_type, a->ring_size, a->queue_priority, a->queue_percentage, a->ctx_save_restore_size,
                  a->ctl_stack_size, static_cast<unsigned long long>(a->eop_buffer_size), r, {}};
      void* pcs[24];
      const int n = backtrace(pcs, 24);
      for (int i = 1; i < n; ++i) q.stack.push_back(frame(pcs[i]));
      g_queues.push_back(std::move(q));
    } else if (_IOC_NR(request) == 0x20) {
      const auto* a = static_cast<const kfd_ioctl_svm_args*>(arg);
      g_svm_sizes.push_back(a->size);
    }
  }
  return r;
}

namespace {

long rss_kb() {
  std::ifstream f("/proc/self/status");
  std::string k;
  long v = -1;
  while (f >> k) {
    if (k == "VmRSS:") {
      f >> v;
      return v;
    }
    f.ignore(4096, '\n');
  }
  return v;
}

std::string kfd_queue_types() {
  char dir[96];
  std::snprintf(dir, sizeof(dir), "/sys/class/kfd/kfd/proc/%d/queues", static_cast<int>(getpid()));
  std::string o = "[";
  if (DIR* d = opendir(dir)) {
    bool first = true;
    while (dirent* e = readdir(d)) {
      if (e->d_name[0] == '.') continue;
      std::ifstream t(std::string(dir) + "/" + e->d_name + "/type");
      std::string ty;
      t >> ty;
      o += (first ? "\"" : ",\"") + ty + "\"";
      first = false;
    }
    closedir(d);
  }
  return o + "]";
}

std::string esc(const std::string& s) {
  std::string o;
  for (char c : s) o += c == '"' || c == '\\' ? '_' : c;
  return o;
}

struct Snapshot {
  size_t queues = 0, svm = 0;
  int ioctls = 0;
};

Snapshot mark() {
  std::lock_guard<std::mutex> lk(g_mu);
  return {g_queues.size(), g_svm_sizes.size(), g_ioctls};
}

std::string step_json(const char* name, hsa_status_t st, const Snapshot& s0) {
  std::lock_guard<std::mutex> lk(g_mu);
  std::string o = std::string("{\"step\":\"") + name + "\",\"status\":" + std::to_string(st) +
                  ",\"rss_kb\":" + std::to_string(rss_kb()) + ",\"kfd_queues\":" + kfd_queue_types() +
                  ",\"kfd_ioctls\":" + std::to_string(g_ioctls - s0.ioctls) + ",\"svm_sizes\":[";
  for (size_t i = s0.svm; i < g_svm_sizes.size(); ++i)
    o += (i > s0.svm ? "," : "") + std::to_string(g_svm_sizes[i]);
  o += "],\"create_queue\":[";
  for (size_t i = s0.queues; i < g_queues.size(); ++i) {
    const QueueCall& q = g_queues[i];
    char head[256];
    std::snprintf(head, sizeof(head),
                  "%s{\"rc\":%d,\"queue_type\":%u,\"ring_size\":%u,\"priority\":%u,\"percentage\":%u,"
                  "\"cwsr_size\":%u,\"ctl_stack_size\":%u,\"eop_size\":%llu,\"stack\":[",
                  i > s0.queues ? "," : "", q.rc, q.queue_type, q.ring_size, q.priority, q.percentage, q.cwsr_size,
                  q.ctl_stack_size, q.eop_size);
    o += head;
    for (size_t k = 0; k < q.stack.size(); ++k) o += (k ? ",\"" : "\"") + esc(q.stack[k]) + "\"";
    o += "]}";
  }
  return o + "]}";
}

#define FN(name) auto name = reinterpret_cast<decltype(&::name)>(dlsym(lib, #name))

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s CODE_OBJECT [--code-first]\n", argv[0]);
    return 2;
  }
  const bool code_first = argc > 2 && std::strcmp(argv[2], "--code-first") == 0;
  std::ifstream co(argv[1], std::ios::binary);
  const std::string blob((std::istreambuf_iterator<char>(co)), std::istreambuf_iterator<char>());
  void* lib = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!lib) {
    std::printf("{\"ok\":false,\"error\":\"dlopen: %s\"}\n", esc(dlerror()).c_str());
    return 1;
  }
  FN(hsa_init);
  FN(hsa_iterate_agents);
  FN(hsa_agent_get_info);
  FN(hsa_queue_create);
  FN(hsa_code_object_reader_create_from_memory);
  FN(hsa_executable_create_alt);
  FN(hsa_executable_load_agent_code_object);
  FN(hsa_executable_freeze);
  FN(hsa_signal_create);
  FN(hsa_amd_agent_iterate_memory_pools);
  FN(hsa_amd_memory_pool_get_info);
  FN(hsa_amd_memory_pool_allocate);
  std::vector<std::string> steps;
  const long rss0 = rss_kb();
  Snapshot s = mark();
  hsa_status_t st = hsa_init();
  steps.push_back(step_json("hsa_init", st, s));
  hsa_agent_t gpu{};
  hsa_iterate_agents(
      [](hsa_agent_t a, void* d) -> hsa_status_t {
        auto* p = static_cast<std::pair<hsa_agent_t*, decltype(hsa_agent_get_info)>*>(d);
        hsa_device_type_t t;
        p->second(a, HSA_AGENT_INFO_DEVICE, &t);
        if (t == HSA_DEVICE_TYPE_GPU && p->first->handle == 0) *p->first = a;
        return HSA_STATUS_SUCCESS;
      },
      new std::pair<hsa_agent_t*, decltype(hsa_agent_get_info)>(&gpu, hsa_agent_get_info));
  if (!gpu.handle) {
    std::printf("{\"ok\":false,\"error\":\"no GPU agent\"}\n");
    return 1;
  }
  hsa_queue_t* q1 = nullptr;
  auto queue_step = [&](const char* name) {
    Snapshot s0 = mark();
    hsa_queue_t* q = nullptr;
    const hsa_status_t r = hsa_queue_create(gpu, 64, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q);
    steps.push_back(step_json(name, r, s0));
    return q;
  };
  auto code_step = [&] {
    Snapshot s0 = mark();
    hsa_code_object_reader_t rd{};
    hsa_executable_t ex{};
    hsa_status_t r = hsa_code_object_reader_create_from_memory(blob.data(), blob.size(), &rd);
    if (r == HSA_STATUS_SUCCESS)
      r = hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &ex);
    if (r == HSA_STATUS_SUCCESS) r = hsa_executable_load_agent_code_object(ex, gpu, rd, nullptr, nullptr);
    if (r == HSA_STATUS_SUCCESS) r = hsa_executable_freeze(ex, nullptr);
    steps.push_back(step_json("code_object_load_freeze", r, s0));
  };
  if (code_first) {
    code_step();
    q1 = queue_step("hsa_queue_create");
  } else {
    q1 = queue_step("hsa_queue_create");
    code_step();
  }
  {
    Snapshot s0 = mark();
    hsa_signal_t sig{};
    hsa_status_t r = hsa_signal_create(1, 0, nullptr, &sig);
    // a kernarg-style allocation in the first system pool that allows kernargs
    struct Ctx {
      decltype(hsa_amd_memory_pool_get_info) info;
      hsa_amd_memory_pool_t pool;
      bool found;
    } c{hsa_amd_memory_pool_get_info, {}, false};
    hsa_agent_t cpu{};
    hsa_iterate_agents(
        [](hsa_agent_t a, void* d) -> hsa_status_t {
          auto* p = static_cast<std::pair<hsa_agent_t*, decltype(hsa_agent_get_info)>*>(d);
          hsa_device_type_t t;
          p->second(a, HSA_AGENT_INFO_DEVICE, &t);
          if (t == HSA_DEVICE_TYPE_CPU && p->first->handle == 0) *p->first = a;
          return HSA_STATUS_SUCCESS;
        },
        new std::pair<hsa_agent_t*, decltype(hsa_agent_get_info)>(&cpu, hsa_agent_get_info));
    hsa_amd_agent_iterate_memory_pools(
        cpu,
        [](hsa_amd_memory_pool_t p, void* d) -> hsa_status_t {
          auto* c = static_cast<Ctx*>(d);
          uint32_t flags = 0;
          c->info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
          if (!c->found && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT)) {
            c->pool = p;
            c->found = true;
          }
          return HSA_STATUS_SUCCESS;
        },
        &c);
    void* kernarg = nullptr;
    if (r == HSA_STATUS_SUCCESS && c.found) r = hsa_amd_memory_pool_allocate(c.pool, 4096, 0, &kernarg);
    steps.push_back(step_json("signal_and_kernarg", r, s0));
  }
  queue_step("second_hsa_queue_create");
  std::string o = "{\"ok\":true,\"order\":\"" + std::string(code_first ? "code-first" : "queue-first") +
                  "\",\"rss_kb_start\":" + std::to_string(rss0) + ",\"steps\":[";
  for (size_t i = 0; i < steps.size(); ++i) o += (i ? "," : "") + steps[i];
  std::printf("%s]}\n", o.c_str());
  std::fflush(stdout);
  _exit(0);  // skip ROCr teardown (not under test)
}
