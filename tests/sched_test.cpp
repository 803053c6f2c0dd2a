// sched_test.cpp -- unit tests of p1_amd/host/scheduler.hpp (the server's job
// policy; server.go:83-168 + handout 4.2), built and run by
// tests/test_server.py::test_scheduler_unit.  Exit status 0 = all passed.
#include <stdio.h>
#include <stdlib.h>

#include "../p1_amd/host/scheduler.hpp"

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      exit(1);                                                     \
    }                                                              \
  } while (0)

static void full_u64_range_is_o1() {
  sched::Scheduler S(1ull << 32);
  const uint64_t id = S.Submit(7, "bradfitz", 0, UINT64_MAX);
  S.AddMiner(1);
  S.AddMiner(2);
  auto a = S.Dispatch();
  CHECK(a.size() == 2);
  CHECK(a[0].lo == 0 && a[0].hi == (1ull << 32) - 1);
  CHECK(a[1].lo == (1ull << 32) && a[1].hi == (2ull << 32) - 1);
  CHECK(S.HeldSpans(id) == 0);  // the rest of the range is one cursor
  // the last chunk ends exactly at 2^64-1 without wrapping
  sched::Scheduler T(1ull << 63);
  const uint64_t t = T.Submit(1, "m", 1, UINT64_MAX);
  T.AddMiner(1);
  auto b = T.Dispatch();
  CHECK(b.size() == 1 && b[0].lo == 1 && b[0].hi == (1ull << 63));
  CHECK(T.Result(1, 5, 9));
  b = T.Dispatch();
  CHECK(b.size() == 1 && b[0].lo == (1ull << 63) + 1 && b[0].hi == UINT64_MAX);
  CHECK(T.Result(1, 4, 10));
  CHECK(T.Dispatch().empty());
  auto d = T.TakeDone();
  CHECK(d.size() == 1 && d[0].req == t && d[0].hash == 4 && d[0].nonce == 10);
}

static void lost_miner_chunk_goes_first() {
  sched::Scheduler S(100);
  const uint64_t id = S.Submit(1, "x", 0, 999);
  S.AddMiner(1);
  S.AddMiner(2);
  auto a = S.Dispatch();  // miner 1: [0,99], miner 2: [100,199]
  CHECK(a.size() == 2 && a[0].miner == 1 && a[0].lo == 0 && a[1].lo == 100);
  S.LoseMiner(1);          // [0,99] goes back to the front
  CHECK(S.HeldSpans(id) == 1);
  S.AddMiner(3);
  a = S.Dispatch();
  CHECK(a.size() == 1 && a[0].miner == 3 && a[0].lo == 0 && a[0].hi == 99);
  CHECK(S.Result(2, 50, 150));
  a = S.Dispatch();
  CHECK(a.size() == 1 && a[0].miner == 2 && a[0].lo == 200 && a[0].hi == 299);  // then the cursor
}

static void answer_and_identity() {
  sched::Scheduler S(10);
  const uint64_t e = S.Submit(1, "x", 5, 3);  // empty range: (MaxUint64, 0) at once
  const uint64_t r = S.Submit(2, "y", 0, 25);
  S.AddMiner(1);
  auto d = S.TakeDone();
  CHECK(d.size() == 1 && d[0].req == e && d[0].hash == UINT64_MAX && d[0].nonce == 0);
  uint64_t hashes[3] = {70, 40, 40};  // a tie across chunks: lowest nonce wins
  uint64_t nonces[3] = {3, 17, 22};
  for (int i = 0; i < 3; ++i) {
    auto a = S.Dispatch();
    CHECK(a.size() == 1 && a[0].req == r);
    CHECK(S.Result(1, hashes[i], nonces[i]));
  }
  d = S.TakeDone();
  CHECK(d.size() == 1 && d[0].hash == 40 && d[0].nonce == 17);
  CHECK(S.Idle());
}

static void completion_order() {
  sched::Scheduler S(1000);
  const uint64_t big = S.Submit(1, "a", 0, 2999);   // 3 chunks
  const uint64_t small = S.Submit(2, "b", 0, 999);  // 1 chunk
  S.AddMiner(1);
  S.AddMiner(2);
  auto a = S.Dispatch();  // round-robin: miner 1 <- big[0], miner 2 <- small
  CHECK(a.size() == 2 && a[0].req == big && a[1].req == small);
  CHECK(S.Result(2, 1, 1));  // small completes first
  CHECK(S.Result(1, 2, 2));
  for (int i = 0; i < 2; ++i) {
    a = S.Dispatch();
    for (auto& x : a) CHECK(S.Result(x.miner, 3, 3));
  }
  auto d = S.TakeDone();
  CHECK(d.size() == 2 && d[0].req == small && d[1].req == big);
}

static void cancelled_client() {
  sched::Scheduler S(10);
  S.Submit(9, "x", 0, UINT64_MAX);
  const uint64_t keep = S.Submit(8, "y", 0, 9);
  S.AddMiner(1);
  auto a = S.Dispatch();
  S.CancelClient(9);
  CHECK(S.Result(a[0].miner, 1, 1));  // a result for a dropped request is absorbed
  a = S.Dispatch();
  CHECK(a.size() == 1 && a[0].req == keep);
  CHECK(S.Result(1, 5, 5));
  auto d = S.TakeDone();
  CHECK(d.size() == 1 && d[0].req == keep);
  CHECK(S.Idle());
}

// A lost miner's in-flight chunk is re-queued at the front and goes to the
// next idle miner.
static void lost_chunk_in_flight() {
  sched::Scheduler S(10);
  const uint64_t id = S.Submit(1, "m", 0, 19);
  S.AddMiner(1);
  S.AddMiner(2);
  auto a = S.Dispatch();
  CHECK(a.size() == 2 && a[0].lo == 0 && a[1].lo == 10);
  CHECK(S.InFlight(id, 0) && S.InFlight(id, 10));
  S.LoseMiner(1);
  CHECK(!S.InFlight(id, 0) && S.HeldSpans(id) == 1);
  CHECK(S.Dispatch().empty());  // miner 2 is still busy
  CHECK(S.Result(2, 9, 12));
  a = S.Dispatch();
  CHECK(a.size() == 1 && a[0].miner == 2 && a[0].lo == 0 && a[0].hi == 9);
  CHECK(S.Result(2, 2, 3));
  CHECK(S.Result(2, 1, 1) == false);  // a stray Result from an idle miner is ignored
  auto d = S.TakeDone();
  CHECK(d.size() == 1 && d[0].hash == 2 && d[0].nonce == 3);
}

int main() {
  full_u64_range_is_o1();
  lost_miner_chunk_goes_first();
  answer_and_identity();
  completion_order();
  cancelled_client();
  lost_chunk_in_flight();
  printf("sched_test: ok\n");
  return 0;
}
