// Randomized model-based simulation of the server's scheduler
// (p1_amd/host/scheduler.hpp; server.go:83-168 + p1.pdf 4.2 splitting,
// fairness and failure handling).
//
//   sched_sim <seed> <rounds>
//
// Clients submit ranges (small enough to brute-force, some at the top of the
// u64 range, some empty), miners join and vanish at random -- some while
// holding a chunk, some after computing it but before reporting -- clients
// go away, idle miners send stray Results, and chunk results arrive in a
// random order.  Each miner "hashes" with a cheap stand-in (splitmix64 of
// the nonce and the message) and reports its chunk's first minimum, as
// miner.go:56-63 does.  Checked on every step:
//   - no nonce is out with two miners at once, and every assignment lies in
//     its request's range;
//   - a request completes at most once, never after its client is gone, and
//     its answer equals the brute-force first minimum of the whole range
//     with miner.go:56's identity;
//   - while at least one miner is alive, every live request completes
//     (the run drains at the end with a fresh miner);
//   - handed-back chunks held per request stay bounded by the losses.
// Prints "sched_sim: ok <requests> <chunks> <losses>" or exits 1.
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>

#include <map>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "../p1_amd/host/scheduler.hpp"

namespace {

uint64_t mix(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}
uint64_t fake_hash(const std::string& d, uint64_t nonce) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : d) h = (h ^ c) * 1099511628211ull;
  const uint64_t v = mix(nonce ^ h);
  // 1 in 16 hashes is MaxUint64; the value range depends on the message,
  // from 2^56 down to 2^9, so some messages have many equal minima (the
  // lowest nonce must win, within a chunk and across chunks)
  return (v & 0xF) == 0 ? UINT64_MAX : v >> (8 + h % 48);
}
// miner.go:56-63 over [lo, hi] (inclusive, no wrap at 2^64-1)
void scan(const std::string& d, uint64_t lo, uint64_t hi, uint64_t* h, uint64_t* n) {
  uint64_t best = UINT64_MAX, bi = 0;
  for (uint64_t i = lo;; ++i) {
    const uint64_t r = fake_hash(d, i);
    if (r < best) { best = r; bi = i; }
    if (i == hi) break;
  }
  *h = best;
  *n = bi;
}

#define FAIL(...)                       \
  do {                                  \
    fprintf(stderr, "sched_sim: ");     \
    fprintf(stderr, __VA_ARGS__);       \
    fprintf(stderr, "\n");              \
    exit(1);                            \
  } while (0)

struct ReqInfo {
  int64_t client;
  std::string data;
  uint64_t lo, hi;
  bool done = false;
};
struct Held {  // a chunk a miner holds (maybe computed, not reported yet)
  uint64_t req, lo, hi;
  bool computed = false;
  uint64_t h = 0, n = 0;
};

}  // namespace

int main(int argc, char** argv) {
  const uint64_t seed = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1;
  const int rounds = argc > 2 ? atoi(argv[2]) : 2000;
  std::mt19937_64 g(seed);
  auto rnd = [&](uint64_t n) { return (uint64_t)(g() % n); };
  const uint64_t chunk = 1 + rnd(3) * 400 + rnd(400);
  sched::Scheduler S(chunk);
  std::map<uint64_t, ReqInfo> reqs;
  std::set<int64_t> gone_clients;
  std::map<int, Held> held;  // busy miners
  std::set<int> miners;
  int next_miner = 1;
  int64_t next_client = 1000000;
  long chunks = 0, losses = 0, completed = 0;

  auto check_done = [&]() {
    for (const sched::Done& d : S.TakeDone()) {
      auto it = reqs.find(d.req);
      if (it == reqs.end()) FAIL("unknown request %" PRIu64 " completed", d.req);
      ReqInfo& r = it->second;
      if (r.done) FAIL("request %" PRIu64 " completed twice", d.req);
      if (gone_clients.count(r.client)) FAIL("request %" PRIu64 " completed after its client left", d.req);
      if (d.client != r.client) FAIL("request %" PRIu64 " answered to the wrong client", d.req);
      uint64_t h = UINT64_MAX, n = 0;
      if (r.lo <= r.hi) scan(r.data, r.lo, r.hi, &h, &n);
      if (h == UINT64_MAX) n = 0;  // miner.go:56 identity
      if (d.hash != h || d.nonce != n)
        FAIL("request %" PRIu64 " [%" PRIu64 ", %" PRIu64 "]: got (%" PRIu64 ", %" PRIu64 ") want (%" PRIu64
             ", %" PRIu64 ")", d.req, r.lo, r.hi, d.hash, d.nonce, h, n);
      r.done = true;
      ++completed;
    }
  };
  auto dispatch = [&]() {
    for (const sched::Assignment& a : S.Dispatch()) {
      auto it = reqs.find(a.req);
      if (it == reqs.end()) FAIL("assignment for unknown request");
      const ReqInfo& r = it->second;
      if (a.lo > a.hi || a.lo < r.lo || a.hi > r.hi || a.hi - a.lo >= chunk || a.data != r.data)
        FAIL("bad assignment [%" PRIu64 ", %" PRIu64 "] for [%" PRIu64 ", %" PRIu64 "]", a.lo, a.hi, r.lo, r.hi);
      if (held.count(a.miner)) FAIL("miner %d given a second chunk", a.miner);
      for (const auto& kv : held)  // no nonce out twice
        if (kv.second.req == a.req && !(a.hi < kv.second.lo || kv.second.hi < a.lo))
          FAIL("overlapping chunks of request %" PRIu64, a.req);
      held[a.miner] = {a.req, a.lo, a.hi};
      ++chunks;
    }
  };
  auto lose = [&](int m) {
    S.LoseMiner(m);
    if (held.count(m)) ++losses;
    held.erase(m);
    miners.erase(m);
  };

  for (int step = 0; step < rounds; ++step) {
    const uint64_t ev = rnd(100);
    if (ev < 12) {  // a client request
      ReqInfo r;
      r.client = rnd(4) == 0 && !reqs.empty() ? reqs.rbegin()->second.client : next_client++;
      if (gone_clients.count(r.client)) r.client = next_client++;
      r.data = std::string(1 + rnd(5), (char)('a' + rnd(26)));
      const uint64_t span = rnd(5) == 0 ? 0 : rnd(6000);
      const uint64_t kind = rnd(10);
      if (kind == 0) { r.hi = UINT64_MAX; r.lo = UINT64_MAX - span; }         // the u64 top
      else if (kind == 1) { r.lo = 100 + rnd(1000); r.hi = r.lo - 1 - rnd(50); }  // lower > upper
      else { r.lo = rnd(1ull << 40); r.hi = r.lo + span; }
      const uint64_t id = S.Submit(r.client, r.data, r.lo, r.hi);
      reqs[id] = r;
    } else if (ev < 20) {  // a miner joins
      const int m = next_miner++;
      S.AddMiner(m);
      miners.insert(m);
    } else if (ev < 24 && !miners.empty()) {  // a miner vanishes (maybe holding a chunk)
      auto it = miners.begin();
      std::advance(it, rnd(miners.size()));
      lose(*it);
    } else if (ev < 27 && !reqs.empty()) {  // a client goes away
      auto it = reqs.begin();
      std::advance(it, rnd(reqs.size()));
      if (!it->second.done) {
        const int64_t c = it->second.client;
        S.CancelClient(c);
        gone_clients.insert(c);
      }
    } else if (ev < 30 && !miners.empty()) {  // a stray Result from an idle miner
      auto it = miners.begin();
      std::advance(it, rnd(miners.size()));
      if (!held.count(*it) && S.Result(*it, g(), g())) FAIL("stray Result accepted");
    } else if (!held.empty()) {  // a busy miner computes, or reports a computed chunk
      auto it = held.begin();
      std::advance(it, rnd(held.size()));
      Held& c = it->second;
      const auto r = reqs.find(c.req);
      if (!c.computed) {
        scan(r->second.data, c.lo, c.hi, &c.h, &c.n);
        if (c.h == UINT64_MAX) c.n = 0;
        c.computed = true;
      } else {
        const int m = it->first;
        const Held done = c;
        held.erase(it);
        if (!S.Result(m, done.h, done.n)) FAIL("Result of a held chunk refused");
      }
    }
    dispatch();
    check_done();
    for (const auto& kv : reqs)
      if (!kv.second.done && S.HeldSpans(kv.first) > (size_t)losses + 1) FAIL("handed-back chunks unbounded");
  }
  // drain: one fresh miner that never fails
  const int m = next_miner++;
  S.AddMiner(m);
  miners.insert(m);
  for (int guard = 0; guard < 10000000; ++guard) {
    dispatch();
    if (held.empty()) break;
    for (auto it = held.begin(); it != held.end();) {
      Held c = it->second;
      const auto r = reqs.find(c.req);
      if (!c.computed) scan(r->second.data, c.lo, c.hi, &c.h, &c.n);
      if (c.h == UINT64_MAX) c.n = 0;
      const int who = it->first;
      it = held.erase(it);
      if (!S.Result(who, c.h, c.n)) FAIL("Result refused while draining");
    }
    check_done();
  }
  check_done();
  long open = 0;
  for (const auto& kv : reqs)
    if (!kv.second.done && !gone_clients.count(kv.second.client)) ++open;
  if (open) FAIL("%ld live requests never completed", open);
  if (!S.Idle()) {
    // only requests of departed clients may remain in no form: CancelClient erased them
    FAIL("scheduler not idle after the drain");
  }
  printf("sched_sim: ok %ld %ld %ld\n", completed, chunks, losses);
  return 0;
}
