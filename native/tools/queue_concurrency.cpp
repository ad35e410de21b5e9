// mi355x-queue-concurrency: do kfd queue creations in ONE process serialise?
// (measurement tool, not shipped)
//
// A pod-mode container with N GPUs creates 2N queues (its own + ROCr's
// internal one per GPU, profiles/archive/measurements_r1_r3.md §3f); each is ~3.7 ms of
// AMDKFD_IOC_SVM (the 181 MB CWSR area) + 1 ms of CREATE_QUEUE. The SVM call
// takes the process' mmap lock and CREATE_QUEUE the process-wide kfd mutex,
// so N threads creating queues on N GPUs would run one after another. On a
// 1-GPU box the same locks are exercised by T threads each creating one queue
// on GPU 0: this tool times that (after a warm-up queue, so ROCr's internal
// queue already exists), and prints CLOCK_MONOTONIC start/end stamps so a
// driver can also compare T separate processes doing one queue each.
//
//   mi355x-queue-concurrency --threads T [--barrier-ns ABS_MONOTONIC_NS] -> one JSON line
#include <dlfcn.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <time.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<uint64_t>(ts.tv_sec) * 1000000000ull + static_cast<uint64_t>(ts.tv_nsec);
}

#define FN(name) decltype(&::name) name = reinterpret_cast<decltype(&::name)>(dlsym(lib, #name))

}  // namespace

int main(int argc, char** argv) {
  int threads = 1;
  uint64_t barrier_ns = 0;
  for (int i = 1; i + 1 < argc; ++i) {
    if (!std::strcmp(argv[i], "--threads")) threads = std::atoi(argv[i + 1]);
    if (!std::strcmp(argv[i], "--barrier-ns")) barrier_ns = std::strtoull(argv[i + 1], nullptr, 10);
  }
  if (threads < 1 || threads > 64) {
    std::printf("{\"ok\":false,\"error\":\"--threads must be 1..64\"}\n");
    return 2;
  }
  void* lib = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!lib) lib = dlopen("/opt/rocm/lib/libhsa-runtime64.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!lib) {
    std::printf("{\"ok\":false,\"error\":\"dlopen failed\"}\n");
    return 2;
  }
  FN(hsa_init);
  FN(hsa_iterate_agents);
  FN(hsa_agent_get_info);
  FN(hsa_queue_create);
  FN(hsa_queue_destroy);
  FN(hsa_shut_down);
  if (hsa_init() != HSA_STATUS_SUCCESS) {
    std::printf("{\"ok\":false,\"error\":\"hsa_init\"}\n");
    return 1;
  }
  struct Ctx {
    hsa_agent_t gpu{};
    bool found = false;
    decltype(&::hsa_agent_get_info) info;
  } c;
  c.info = hsa_agent_get_info;
  hsa_iterate_agents(
      [](hsa_agent_t a, void* p) {
        auto* c = static_cast<Ctx*>(p);
        hsa_device_type_t t;
        c->info(a, HSA_AGENT_INFO_DEVICE, &t);
        if (t == HSA_DEVICE_TYPE_GPU && !c->found) c->gpu = a, c->found = true;
        return HSA_STATUS_SUCCESS;
      },
      &c);
  if (!c.found) {
    std::printf("{\"ok\":false,\"error\":\"no GPU agent\"}\n");
    return 1;
  }
  // warm-up queue: ROCr creates its internal queue here, not inside the timed part
  hsa_queue_t* warm = nullptr;
  const uint64_t w0 = mono_ns();
  if (hsa_queue_create(c.gpu, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &warm) !=
      HSA_STATUS_SUCCESS) {
    std::printf("{\"ok\":false,\"error\":\"warm-up queue\"}\n");
    return 1;
  }
  const double warm_ms = (mono_ns() - w0) / 1e6;
  while (barrier_ns && mono_ns() < barrier_ns) {
  }
  std::vector<hsa_queue_t*> qs(threads, nullptr);
  std::vector<uint64_t> t0(threads), t1(threads);
  std::atomic<int> ready{0}, bad{0};
  std::atomic<bool> go{false};
  std::vector<std::thread> th;
  for (int i = 0; i < threads; ++i)
    th.emplace_back([&, i] {
      ready.fetch_add(1);
      while (!go.load()) {
      }
      t0[i] = mono_ns();
      if (hsa_queue_create(c.gpu, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &qs[i]) !=
          HSA_STATUS_SUCCESS)
        bad.fetch_add(1);
      t1[i] = mono_ns();
    });
  while (ready.load() < threads) {
  }
  const uint64_t start = mono_ns();
  go.store(true);
  for (auto& t : th) t.join();
  uint64_t end = 0;
  double sum_ms = 0;
  std::string per = "[";
  for (int i = 0; i < threads; ++i) {
    end = t1[i] > end ? t1[i] : end;
    const double ms = (t1[i] - t0[i]) / 1e6;
    sum_ms += ms;
    per += (i ? "," : "") + std::to_string(ms);
  }
  per += "]";
  std::printf("{\"ok\":%s,\"threads\":%d,\"warmup_queue_ms\":%.3f,\"wall_ms\":%.3f,\"sum_ms\":%.3f,"
              "\"start_ns\":%llu,\"end_ns\":%llu,\"per_queue_ms\":%s}\n",
              bad.load() ? "false" : "true", threads, warm_ms, (end - start) / 1e6, sum_ms,
              static_cast<unsigned long long>(start), static_cast<unsigned long long>(end), per.c_str());
  std::fflush(stdout);
  for (auto* q : qs)
    if (q) hsa_queue_destroy(q);
  hsa_queue_destroy(warm);
  hsa_shut_down();
  return bad.load() ? 1 : 0;
}
