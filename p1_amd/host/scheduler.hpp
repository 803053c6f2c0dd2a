// scheduler.hpp -- the bitcoin server's job bookkeeping, independent of the
// transport that carries requests and results (LSP connections in
// `p1server lsp`, child-process pipes in `p1server scan|serve`).
//
// Reference: /root/reference/src/github.com/cmu440/bitcoin/server/server.go
//   :119-140  a client Request is handed, unsplit, to the first idle miner
//   :141-152  a miner's Result is forwarded to the requesting client
//   :86-115   a lost miner's job should go to another miner (buggy there:
//             it writes to the lost connection and re-queues the job twice)
//   :153-167  a Join makes a miner idle and hands it the oldest queued job
// The handout (p1.pdf 4.2) asks the server to split large requests over the
// miners, to schedule fairly and to survive miner and client loss.  Here:
//   * a request [Lower, Upper] is carved into chunks of at most `chunk`
//     nonces on demand: it holds only a cursor (next unsent nonce, Upper) and
//     a short queue of chunks handed back by lost miners, so its memory is
//     O(1) in the range size -- client.go:21 accepts any uint64 maxNonce and
//     server.go:119-140 forwards any range, so [0, 2^64-1] must be cheap;
//   * idle miners take chunks round-robin over the open requests, so a small
//     request is not starved behind a large one;
//   * a lost miner's chunk goes back to the front of its request's queue;
//   * a lost client's requests are dropped (results of their chunks still in
//     flight are ignored when they arrive);
//   * a request's answer is the lexicographic (hash, nonce) min over its
//     chunks with miner.go:56's identity (MaxUint64, 0) -- identical to one
//     miner scanning the whole range (contiguous chunks, strict '<');
// (Round 3 had opt-in tail hedging -- idle miners running copies of the
// chunks in flight longest -- against the one-epoch resend stall at 5% loss.
// Sending each first transmission 3 times (lsp::Params::Copies) removed the
// stall, after which hedging measured as a pure loss: 8 miners on one GPU,
// configs[4], 2.64 s against 1.89 s median (profiles/r04b_lsp_m8c3h.json,
// r04b_lsp_m8c3.json).  It was removed in round 4.)
#pragma once
#include <stdint.h>

#include <deque>
#include <map>
#include <string>
#include <vector>

namespace sched {

struct Assignment {
  int miner;
  uint64_t req;
  std::string data;
  uint64_t lo, hi;
};

struct Done {
  uint64_t req;
  int64_t client;  // transport key of the requester
  uint64_t hash, nonce;
};

class Scheduler {
 public:
  explicit Scheduler(uint64_t chunk) : chunk_(chunk ? chunk : (1ull << 32)) {}

  // A client request (server.go:119-140, with splitting).  Returns its id.
  uint64_t Submit(int64_t client, const std::string& data, uint64_t lo, uint64_t hi) {
    Req r;
    r.id = next_id_++;
    r.client = client;
    r.data = data;
    r.next = lo;
    r.hi = hi;
    r.exhausted = lo > hi;  // an empty range is answered at once (identity)
    order_.push_back(r.id);
    const uint64_t id = r.id;
    reqs_.emplace(id, std::move(r));
    if (lo > hi) done_.push_back(id);
    return id;
  }

  // The requester's connection is gone: forget its requests.
  void CancelClient(int64_t client) {
    for (auto it = reqs_.begin(); it != reqs_.end();) {
      if (it->second.client == client) {
        drop_order(it->first);
        it = reqs_.erase(it);
      } else {
        ++it;
      }
    }
  }

  void AddMiner(int miner) { miners_[miner]; }  // idle (server.go:153-166)
  bool IsMiner(int miner) const { return miners_.count(miner) != 0; }
  size_t Miners() const { return miners_.size(); }

  // A miner is lost: its chunk goes back to the front of its request
  // (unless the request is gone).
  void LoseMiner(int miner) {
    auto it = miners_.find(miner);
    if (it == miners_.end()) return;
    const Miner& m = it->second;
    if (m.busy) {
      auto r = reqs_.find(m.cur_req);
      if (r != reqs_.end()) {
        auto f = r->second.inflight.find(m.lo);
        if (f != r->second.inflight.end()) {
          r->second.inflight.erase(f);
          r->second.back.push_front({m.lo, m.hi});
        }
      }
    }
    miners_.erase(it);
  }

  // A miner's Result for its current chunk.  Returns false if the miner had
  // no chunk (a stray Result is ignored).
  bool Result(int miner, uint64_t hash, uint64_t nonce) {
    auto it = miners_.find(miner);
    if (it == miners_.end() || !it->second.busy) return false;
    Miner& m = it->second;
    m.busy = false;
    auto r = reqs_.find(m.cur_req);
    if (r == reqs_.end()) return true;  // its client is gone
    Req& q = r->second;
    auto f = q.inflight.find(m.lo);
    if (f == q.inflight.end()) return true;  // not (or no longer) outstanding
    q.inflight.erase(f);
    if (!q.has_work() && q.inflight.empty()) done_.push_back(q.id);
    // a chunk whose hashes are all MaxUint64 reports (Max, 0); only real
    // minima (< Max) take part, lexicographically -- identity of miner.go:56
    if (hash < UINT64_MAX && (!q.found || hash < q.best || (hash == q.best && nonce < q.best_n))) {
      q.best = hash;
      q.best_n = nonce;
      q.found = true;
    }
    return true;
  }

  // Hand one chunk to every idle miner, round-robin over open requests.
  std::vector<Assignment> Dispatch() {
    std::vector<Assignment> out;
    for (auto& kv : miners_) {
      Miner& m = kv.second;
      if (m.busy) continue;
      bool any = false;
      for (size_t tries = 0; tries < order_.size(); ++tries) {
        const uint64_t id = order_[rr_++ % order_.size()];
        auto it = reqs_.find(id);
        if (it == reqs_.end() || !it->second.has_work()) continue;
        Req& r = it->second;
        const Span c = r.take(chunk_);
        r.inflight[c.lo] = {c.hi};
        assign(kv.first, m, r, c.lo, c.hi, out);
        any = true;
        break;
      }
      if (!any) break;
    }
    return out;
  }

  // A chunk could not be sent (the miner's connection failed): undo it and
  // drop the miner.
  void Unassign(int miner) { LoseMiner(miner); }

  // Requests whose chunks are all answered, in the order they completed.
  std::vector<Done> TakeDone() {
    std::vector<Done> out;
    for (uint64_t id : done_) {
      auto it = reqs_.find(id);
      if (it == reqs_.end()) continue;  // its client went away meanwhile
      const Req& r = it->second;
      out.push_back({r.id, r.client, r.found ? r.best : UINT64_MAX, r.found ? r.best_n : 0});
      drop_order(r.id);
      reqs_.erase(it);
    }
    done_.clear();
    return out;
  }

  // The chunk of `req` that starts at `lo` is out with a miner and not
  // answered yet.  Tests use it.
  bool InFlight(uint64_t req, uint64_t lo) const {
    auto it = reqs_.find(req);
    return it != reqs_.end() && it->second.inflight.count(lo) != 0;
  }

  // Chunks a request still holds in memory (handed-back chunks; the unsent
  // rest of its range is one cursor).  Tests bound this.
  size_t HeldSpans(uint64_t req) const {
    auto it = reqs_.find(req);
    return it == reqs_.end() ? 0 : it->second.back.size();
  }

  bool Idle() const { return reqs_.empty(); }
  // Work is waiting but no miner could take it.
  bool Starved() const { return !reqs_.empty() && miners_.empty(); }

 private:
  struct Span {
    uint64_t lo, hi;
  };
  struct Flight {     // a chunk sent to a miner, not answered yet
    uint64_t hi;
  };
  struct Req {
    uint64_t id;
    int64_t client;
    std::string data;
    std::deque<Span> back;       // chunks handed back by lost miners (sent first)
    uint64_t next = 0, hi = 0;   // cursor: [next, hi] not handed out yet
    bool exhausted = false;      // the cursor has passed hi
    std::map<uint64_t, Flight> inflight;  // by chunk lo
    uint64_t best = UINT64_MAX, best_n = 0;
    bool found = false;
    bool has_work() const { return !back.empty() || !exhausted; }
    // next chunk: a handed-back one, else carved from the cursor
    Span take(uint64_t chunk) {
      if (!back.empty()) {
        const Span c = back.front();
        back.pop_front();
        return c;
      }
      const uint64_t b = (hi - next >= chunk) ? next + (chunk - 1) : hi;
      const Span c{next, b};
      if (b == hi) exhausted = true;  // no wrap at 2^64-1
      else next = b + 1;
      return c;
    }
  };
  struct Miner {
    bool busy = false;
    uint64_t cur_req = 0, lo = 0, hi = 0;
  };

  static void assign(int id, Miner& m, const Req& r, uint64_t lo, uint64_t hi, std::vector<Assignment>& out) {
    m.busy = true;
    m.cur_req = r.id;
    m.lo = lo;
    m.hi = hi;
    out.push_back({id, r.id, r.data, lo, hi});
  }
  void drop_order(uint64_t id) {
    for (size_t i = 0; i < order_.size(); ++i)
      if (order_[i] == id) {
        order_.erase(order_.begin() + i);
        return;
      }
  }

  uint64_t chunk_;
  std::map<int, Miner> miners_;
  std::map<uint64_t, Req> reqs_;
  std::vector<uint64_t> order_;
  std::vector<uint64_t> done_;  // completed request ids, in completion order
  size_t rr_ = 0;
  uint64_t next_id_ = 1;
};

}  // namespace sched
