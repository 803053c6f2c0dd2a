// The library's host runtime (p1_amd/csrc/p1hip.hip: planner, launches,
// device threads, combine, error paths) under AddressSanitizer +
// UndefinedBehaviorSanitizer, driving real scans on the GPU.  Only the host
// code is instrumented (`make sanitize-lib`: -Xarch_host -fsanitize=...);
// the kernels are the shipped code object, unchanged.
//
//   capi_san_stress <seconds>
//
// Phases (each prints one line; any mismatch or unexpected rc exits 1):
//   plan    p1hip_plan_shards on random ranges (host only): n shards, in order,
//           contiguous, covering [lower, upper] exactly
//   args    argument / index errors return their rc and a message
//   scan    random messages (0..200 bytes) x random ranges: small-path sizes,
//           fast-path sizes, decade edges, the top of u64; exact against the
//           oracle up to 3e5 nonces, above that by re-hash + split-min
//   threads 4 host threads calling p1hip_scan / p1hip_hash at once
//   reduce  p1hip_reduce_pairs on crafted arrays (ties, all-UINT64_MAX, n = 0)
//   chaos   4 scanning threads beside a 5th that shuts down / re-opens the
//           library and reads its stats, identity and knobs
//   knobs   P1HIP_TEST_KNOBS paths: 3 logical devices with host combine,
//           multi-launch, MODE 5 table refused (re-plan), small share spans,
//           an injected device failure (rc -2) and recovery
//   reinit  shutdown / init cycles
// Built by tests/test_capi_c.py::test_host_runtime_under_asan (GPU).
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "p1hip.h"

#if defined(__has_feature)
#if __has_feature(address_sanitizer)
#include <sanitizer/lsan_interface.h>
#include <unistd.h>
#define P1_ASAN_BUILD 1
#endif
#endif

extern "C" {
uint64_t p1o_hash(const uint8_t* msg, size_t len, uint64_t nonce);
int p1o_scan_mt(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, int nthreads, uint64_t* out_hash,
                uint64_t* out_nonce);
}

namespace {

using Clock = std::chrono::steady_clock;
std::atomic<int> g_fail{0};

#define CHECK(cond, ...)                                          \
  do {                                                            \
    if (!(cond)) {                                                \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);        \
      fprintf(stderr, __VA_ARGS__);                               \
      fprintf(stderr, " [last_error: %s]\n", p1hip_last_error()); \
      g_fail = 1;                                                 \
      return false;                                               \
    }                                                             \
  } while (0)

std::string rand_msg(std::mt19937_64& g) {
  const int len = std::uniform_int_distribution<int>(0, 200)(g);
  std::string m(len, ' ');
  for (auto& c : m) c = (char)std::uniform_int_distribution<int>(32, 126)(g);
  return m;
}

uint64_t pow10u(int k) {
  uint64_t p = 1;
  while (k-- > 0) p *= 10;
  return p;
}

// a range of `span` nonces around one of: 0, a decade edge, a random point, the u64 top
void rand_range(std::mt19937_64& g, uint64_t span, uint64_t* lo, uint64_t* hi) {
  const int kind = std::uniform_int_distribution<int>(0, 3)(g);
  uint64_t base;
  if (kind == 0) {
    base = 0;
  } else if (kind == 1) {
    const uint64_t edge = pow10u(std::uniform_int_distribution<int>(1, 19)(g));
    base = edge - std::min<uint64_t>(edge, std::uniform_int_distribution<uint64_t>(0, span)(g));
  } else if (kind == 2) {
    base = g() >> std::uniform_int_distribution<int>(0, 40)(g);
  } else {
    base = UINT64_MAX - span + 1 - std::uniform_int_distribution<uint64_t>(0, span)(g) % 3;
  }
  *lo = base;
  *hi = (UINT64_MAX - base < span - 1) ? UINT64_MAX : base + span - 1;
}

bool check_scan(const std::string& m, uint64_t lo, uint64_t hi, int oracle_threads) {
  const uint8_t* p = (const uint8_t*)m.data();
  uint64_t h = 0, n = 0;
  int rc = p1hip_scan(p, m.size(), lo, hi, &h, &n);
  CHECK(rc == P1HIP_OK, "scan rc %d len %zu [%" PRIu64 ", %" PRIu64 "]", rc, m.size(), lo, hi);
  if (hi - lo <= 300000) {
    uint64_t wh = 0, wn = 0;
    p1o_scan_mt(p, m.size(), lo, hi, oracle_threads, &wh, &wn);
    CHECK(h == wh && n == wn, "scan len %zu [%" PRIu64 ", %" PRIu64 "]: got (%" PRIu64 ", %" PRIu64
          ") want (%" PRIu64 ", %" PRIu64 ")", m.size(), lo, hi, h, n, wh, wn);
    return true;
  }
  // too many nonces for the CPU: the answer is a real hash of an in-range
  // nonce, and the min of the two halves (first one on ties) is the same
  CHECK(n >= lo && n <= hi && p1o_hash(p, m.size(), n) == h, "re-hash len %zu nonce %" PRIu64, m.size(), n);
  const uint64_t mid = lo + (hi - lo) / 2;
  uint64_t h1 = 0, n1 = 0, h2 = 0, n2 = 0;
  CHECK(p1hip_scan(p, m.size(), lo, mid, &h1, &n1) == P1HIP_OK, "half 1");
  CHECK(p1hip_scan(p, m.size(), mid + 1, hi, &h2, &n2) == P1HIP_OK, "half 2");
  const bool second = h2 < h1;
  CHECK(h == (second ? h2 : h1) && n == (second ? n2 : n1), "split-min len %zu [%" PRIu64 ", %" PRIu64 "]",
        m.size(), lo, hi);
  return true;
}

bool phase_plan(std::mt19937_64& g, double secs) {
  const auto end = Clock::now() + std::chrono::duration<double>(secs);
  long cases = 0;
  std::vector<uint64_t> first(64), last(64);
  while (Clock::now() < end) {
    const std::string m = rand_msg(g);
    const int n = std::uniform_int_distribution<int>(1, 64)(g);
    uint64_t lo, hi;
    rand_range(g, std::max<uint64_t>(1, g() >> std::uniform_int_distribution<int>(0, 63)(g)), &lo, &hi);
    if (cases % 17 == 0) std::swap(lo, hi);  // lower > upper: n empty shards
    const int rc = p1hip_plan_shards((const uint8_t*)m.data(), m.size(), lo, hi, n, first.data(), last.data());
    CHECK(rc == P1HIP_OK, "plan rc %d", rc);
    if (lo > hi) {
      for (int i = 0; i < n; ++i) CHECK(first[i] > last[i], "plan: lower > upper gives empty shards");
    } else {
      uint64_t next = lo;
      bool done = false;
      for (int i = 0; i < n; ++i) {
        if (first[i] > last[i]) continue;  // empty shard
        CHECK(!done && first[i] == next, "plan: shard %d not contiguous", i);
        if (last[i] == hi) done = true;
        else next = last[i] + 1;
      }
      CHECK(done, "plan: shards do not reach upper");
    }
    ++cases;
  }
  printf("plan ok: %ld random plans\n", cases);
  return true;
}

bool phase_args() {
  uint64_t h = 0, n = 0;
  const uint8_t b = 'x';
  CHECK(p1hip_scan(nullptr, 1, 0, 9, &h, &n) == P1HIP_ERR_ARGS, "NULL msg with len 1");
  CHECK(strlen(p1hip_last_error()) > 0, "no error message");
  // the length is checked before the buffer is read (1 byte really there)
  CHECK(p1hip_scan(&b, P1HIP_MAX_MSG_LEN + 1, 0, 9, &h, &n) == P1HIP_ERR_ARGS, "msg_len over the limit");
  CHECK(p1hip_scan(&b, 1, 0, 9, nullptr, &n) != P1HIP_OK, "NULL out_hash");
  CHECK(p1hip_scan(&b, 1, 9, 0, &h, &n) == P1HIP_OK && h == UINT64_MAX && n == 0, "lower > upper identity");
  CHECK(p1hip_scan(nullptr, 0, 0, 99, &h, &n) == P1HIP_OK, "empty message, NULL pointer, len 0");
  p1hip_device_info_t info;
  CHECK(p1hip_device_info(7, &info) != P1HIP_OK, "device_info bad index");
  CHECK(p1hip_device_info(0, nullptr) != P1HIP_OK, "device_info NULL out");
  p1hip_device_stats_t ds;
  CHECK(p1hip_get_device_stats(-1, &ds) != P1HIP_OK, "device stats bad index");
  std::vector<uint64_t> f(4), l(4);
  CHECK(p1hip_plan_shards(&b, 1, 0, 9, 0, f.data(), l.data()) != P1HIP_OK, "plan n = 0");
  CHECK(p1hip_reduce_pairs(nullptr, nullptr, 5, &h, &n) != P1HIP_OK, "reduce NULL arrays");
  CHECK(p1hip_reduce_pairs(nullptr, nullptr, 0, &h, &n) == P1HIP_OK && h == UINT64_MAX && n == 0, "reduce n = 0");
  // a good call after the errors
  CHECK(p1hip_scan((const uint8_t*)"bradfitz", 8, 0, 9999, &h, &n) == P1HIP_OK && h == 1419516646206828ull &&
            n == 9898, "configs[0] after errors");
  printf("args ok\n");
  return true;
}

bool phase_scan(std::mt19937_64& g, double secs, int oracle_threads, const char* tag,
                uint64_t big = 200000000) {
  const auto end = Clock::now() + std::chrono::duration<double>(secs);
  long cases = 0, nonces = 0;
  auto beat = Clock::now() + std::chrono::seconds(20);
  // exact-checkable sizes most of the time, larger fast-path ranges sometimes
  while (Clock::now() < end && !g_fail) {
    if (Clock::now() > beat) {  // a long run keeps writing (a silent run looks hung)
      printf("%s ... %ld scans\n", tag, cases);
      beat += std::chrono::seconds(20);
    }
    const std::string m = rand_msg(g);
    const int sz = std::uniform_int_distribution<int>(0, 9)(g);
    uint64_t span = sz < 3 ? std::uniform_int_distribution<uint64_t>(1, 70000)(g)
                  : sz < 8 ? std::uniform_int_distribution<uint64_t>(70000, 300000)(g)
                           : std::uniform_int_distribution<uint64_t>(1000000, big)(g);
    uint64_t lo, hi;
    rand_range(g, span, &lo, &hi);
    if (!check_scan(m, lo, hi, oracle_threads)) return false;
    uint64_t h = 0;
    const uint64_t k = lo + (hi - lo) / 3;
    CHECK(p1hip_hash((const uint8_t*)m.data(), m.size(), k, &h) == P1HIP_OK &&
              h == p1o_hash((const uint8_t*)m.data(), m.size(), k), "hash");
    ++cases;
    nonces += (long)(hi - lo + 1);
  }
  printf("%s ok: %ld scans, %ld nonces\n", tag, cases, nonces);
  return !g_fail;
}

bool phase_threads(uint64_t seed, double secs) {
  std::vector<std::thread> ts;
  std::atomic<int> bad{0};
  for (int t = 0; t < 4; ++t)
    ts.emplace_back([&, t] {
      std::mt19937_64 g(seed + 1000 + t);
      if (!phase_scan(g, secs, 2, "thread")) bad = 1;
    });
  for (auto& t : ts) t.join();
  CHECK(!bad, "a thread failed");
  printf("threads ok\n");
  return true;
}

bool phase_reduce(std::mt19937_64& g) {
  for (int it = 0; it < 200; ++it) {
    const size_t n = it < 100 ? std::uniform_int_distribution<size_t>(1, 3000)(g)
                              : std::uniform_int_distribution<size_t>(1, 200000)(g);
    std::vector<uint64_t> hs(n), ns(n);
    const int mode = it % 4;
    for (size_t i = 0; i < n; ++i) {
      hs[i] = mode == 0 ? g() : mode == 1 ? (g() & 7) : mode == 2 ? UINT64_MAX : (UINT64_MAX - (g() & 1));
      ns[i] = g();
    }
    uint64_t wh = UINT64_MAX, wn = 0;  // miner.go:56 identity, lexicographic (hash, nonce) min
    for (size_t i = 0; i < n; ++i)
      if (hs[i] < wh || (hs[i] == wh && hs[i] != UINT64_MAX && ns[i] < wn)) wh = hs[i], wn = ns[i];
    if (wh == UINT64_MAX) wn = 0;
    uint64_t h = 0, nn = 0;
    CHECK(p1hip_reduce_pairs(hs.data(), ns.data(), n, &h, &nn) == P1HIP_OK, "reduce rc");
    CHECK(h == wh && nn == wn, "reduce mode %d n %zu", mode, n);
  }
  printf("reduce ok\n");
  return true;
}

// scans on 4 threads while a 5th shuts the library down, re-opens it and
// reads its stats and identity: every scan must still succeed (a scan after
// a shutdown re-initialises lazily) with the exact answer
bool phase_chaos(uint64_t seed, double secs) {
  std::atomic<bool> stop{false};
  std::atomic<int> bad{0};
  std::atomic<long> cycles{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < 4; ++t)
    ts.emplace_back([&, t] {
      std::mt19937_64 g(seed + 2000 + t);
      long n = 0;
      while (!stop && !bad) {
        const std::string m = rand_msg(g);
        uint64_t lo, hi;
        rand_range(g, std::uniform_int_distribution<uint64_t>(1, 200000)(g), &lo, &hi);
        if (!check_scan(m, lo, hi, 2)) bad = 1;
        ++n;
      }
      printf("chaos thread %d: %ld scans\n", t, n);
    });
  ts.emplace_back([&] {
    std::mt19937_64 g(seed + 3000);
    const int one[1] = {0};
    while (!stop && !bad) {
      switch (g() % 8) {
        case 0: p1hip_shutdown(); break;
        case 1: if (p1hip_init(1, nullptr) != P1HIP_OK) bad = 2; break;
        case 2: if (p1hip_init_devices(one, 1) != P1HIP_OK) bad = 3; break;
        case 3: { p1hip_stats_t st; if (p1hip_get_stats(&st) != P1HIP_OK) bad = 4; break; }
        case 4: p1hip_reset_stats(); break;
        case 5: { p1hip_device_info_t in; (void)p1hip_device_info(0, &in); break; }  // may be closed: rc varies
        case 6: p1hip_set_profiling((int)(g() & 1)); break;
        default: if (strlen(p1hip_test_knobs()) != 0) bad = 5; break;
      }
      ++cycles;
      std::this_thread::sleep_for(std::chrono::milliseconds(g() % 20));
    }
  });
  std::this_thread::sleep_for(std::chrono::duration<double>(secs));
  stop = true;
  for (auto& t : ts) t.join();
  CHECK(!bad, "chaos: failure %d", bad.load());
  // leave the library open on one device for the phases that follow
  p1hip_shutdown();
  CHECK(p1hip_init(1, nullptr) == P1HIP_OK, "chaos: re-init");
  printf("chaos ok: %ld lifecycle calls beside the scans\n", cycles.load());
  return true;
}

void set_knobs(const std::vector<std::pair<const char*, const char*>>& kv) {
  setenv("P1HIP_TEST_KNOBS", "1", 1);
  for (auto& p : kv) setenv(p.first, p.second, 1);
}
void clear_knobs() {
  for (const char* k : {"P1HIP_TEST_KNOBS", "P1HIP_NO_RCCL", "P1HIP_TEST_FAIL_DEVICE", "P1HIP_SMALL_MAX_NONCES",
                        "P1HIP_MAX_LAUNCH_BLOCKS", "P1HIP_KWTAB_MAX_BYTES", "P1HIP_MAX_SCAN_SPAN",
                        "P1HIP_MIN_FAST_THREADS"})
    unsetenv(k);
}

bool phase_knobs(std::mt19937_64& g, double secs) {
  const int three[3] = {0, 0, 0};
  // three logical devices (GPU 0 listed 3x), host combine: device threads,
  // sharding and the two-phase combine under the sanitizer
  set_knobs({{"P1HIP_NO_RCCL", "1"}, {"P1HIP_SMALL_MAX_NONCES", "0"}, {"P1HIP_MIN_FAST_THREADS", "1"}});
  p1hip_shutdown();
  CHECK(p1hip_init_devices(three, 3) == P1HIP_OK && p1hip_device_count() == 3, "3 logical devices");
  if (!phase_scan(g, secs / 3, 8, "knobs/3dev")) return false;
  // per-scan knobs: multi-launch, MODE 5 table refused, small share spans
  set_knobs({{"P1HIP_MAX_LAUNCH_BLOCKS", "3"}, {"P1HIP_KWTAB_MAX_BYTES", "0"}, {"P1HIP_MAX_SCAN_SPAN", "5000"}});
  // (3 workgroups per launch: keep the property-checked ranges small)
  if (!phase_scan(g, secs / 3, 8, "knobs/caps", 3000000)) return false;
  // an injected failure on device 1: every scan fails with rc -2, no hang
  set_knobs({{"P1HIP_TEST_FAIL_DEVICE", "1"}});
  p1hip_shutdown();
  CHECK(p1hip_init_devices(three, 3) == P1HIP_OK, "re-init with a failing device");
  uint64_t h = 0, n = 0;
  for (int i = 0; i < 5; ++i)
    CHECK(p1hip_scan((const uint8_t*)"bradfitz", 8, 0, 999999, &h, &n) == P1HIP_ERR_HIP, "injected failure");
  clear_knobs();
  p1hip_shutdown();
  CHECK(p1hip_init(1, nullptr) == P1HIP_OK, "recover");
  CHECK(p1hip_scan((const uint8_t*)"bradfitz", 8, 0, 9999, &h, &n) == P1HIP_OK && n == 9898, "after recovery");
  printf("knobs ok\n");
  return true;
}

bool phase_reinit(std::mt19937_64& g) {
  const int one[1] = {0};
  for (int i = 0; i < 4; ++i) {
    p1hip_shutdown();
    p1hip_shutdown();  // safe twice
    CHECK((i % 2 ? p1hip_init_devices(one, 1) : p1hip_init(1, nullptr)) == P1HIP_OK, "init %d", i);
    if (!phase_scan(g, 1.0, 8, "reinit")) return false;
  }
  printf("reinit ok\n");
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);  // progress lines reach a log file at once
  const double secs = argc > 1 ? atof(argv[1]) : 30.0;
  const uint64_t seed = argc > 2 ? strtoull(argv[2], nullptr, 10) : 440;
  std::mt19937_64 g(seed);
  clear_knobs();
  if (!phase_plan(g, secs * 0.05)) return 1;
  int got = 0;
  const int rc = p1hip_init(1, &got);
  if (rc == P1HIP_ERR_NO_DEVICE) {
    printf("nodevice %s\n", p1hip_last_error());
    return 0;
  }
  if (rc != P1HIP_OK) {
    fprintf(stderr, "init rc %d: %s\n", rc, p1hip_last_error());
    return 1;
  }
  bool ok = phase_args() && phase_scan(g, secs * 0.25, 8, "scan") && phase_threads(seed, secs * 0.2) &&
            phase_reduce(g) && phase_chaos(seed, secs * 0.1) && phase_knobs(g, secs * 0.25) && phase_reinit(g);
  p1hip_shutdown();
  printf(ok ? "ok\n" : "FAILED\n");
#ifdef P1_ASAN_BUILD
  // Leak-check now, then leave without the ROCm runtime's static
  // destructors: under ROCm's ASan runtime their frees at exit can trip an
  // allocator CHECK ("!dev_runtime_unloaded_", sanitizer_allocator_device.h)
  // after every phase has passed (r04p; DESIGN.md 6 "The r04p teardown
  // abort" has the stack and whose free it is).  P1_SAN_NORMAL_EXIT=1 skips
  // this and returns through the normal exit path, to reproduce it.
  const char* normal = getenv("P1_SAN_NORMAL_EXIT");
  if (!(normal && normal[0] == '1')) {
    fflush(stdout);
    __lsan_do_leak_check();
    _exit(ok ? 0 : 1);
  }
#endif
  return ok ? 0 : 1;
}
