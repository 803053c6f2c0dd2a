// lsp_scenarios -- TEST DRIVER: the reference's LSP test scenarios restated
// against this repository's C++ LSP (p1_amd/host/lsp.{hpp,cpp}), one scenario
// per process run (the fault-injection knobs are process-global).
//
//   lsp_scenarios [--copies K] <name>   exit 0 = pass, 1 = fail (reason on
//                            stderr); --copies sends every first transmission
//                            K times (lsp::Params::Copies, not in the reference)
//   lsp_scenarios --list     names
//
// Scenarios and parameters follow /root/reference/src/github.com/cmu440/lsp:
//   lsp1_test.go:201-335  Basic1-9, SendReceive1-3, Robust1-6 (echo server,
//                         random client payloads, write drop, random delays)
//   lsp2_test.go:476-516  Window1-3 (max capacity: a peer that cannot ack
//                         holds the sender at W messages), Window4-6
//                         (scattered: out-of-order arrival is held back)
//   lsp3_test.go:322-392  ServerSlowStart, ServerClose, ServerCloseConns,
//                         ClientClose
//   lsp4_test.go:444-526  ServerFastClose, ServerToClient, ClientToServer,
//                         RoundTrip (network toggled off/on around buffered
//                         traffic and blocking Close calls)
//   lsp5_test.go:193-203  VariableLengthMsgServer/Client (Size field checks)
// The Go tests' goroutines and channels become std::thread and a small
// blocking queue; their pass/fail conditions are kept.
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../p1_amd/host/lsp.hpp"
#include "../../p1_amd/host/lspnet.hpp"

using namespace std::chrono;

namespace {

std::atomic<bool> g_failed{false};
std::mutex g_log_mu;

void fail(const std::string& why) {
  std::lock_guard<std::mutex> g(g_log_mu);
  if (!g_failed.exchange(true)) fprintf(stderr, "FAIL: %s\n", why.c_str());
}

void sleep_ms(int ms) { std::this_thread::sleep_for(milliseconds(ms)); }

// A failed scenario may leave threads blocked inside LSP calls; end the
// process rather than tear endpoints down under them.
void bail_if_failed(bool ok) {
  if (ok && !g_failed) return;
  fail("scenario failed");
  fflush(stdout);
  fflush(stderr);
  _exit(1);
}

int rnd(int n) {
  thread_local std::mt19937 r(std::random_device{}());
  return n > 0 ? (int)(r() % (unsigned)n) : 0;
}

int g_copies = 1;  // --copies K: Params::Copies of every endpoint (1 = the reference)

lsp::Params P(int limit, int ms, int w) {
  lsp::Params p;
  p.EpochLimit = limit;
  p.EpochMillis = ms;
  p.WindowSize = w;
  p.Copies = g_copies;
  return p;
}

// A blocking queue with a deadline, standing in for Go channels.
template <typename T>
class Chan {
 public:
  void put(T v) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(v));
    }
    cv_.notify_all();
  }
  bool get(T* out, steady_clock::time_point deadline) {
    std::unique_lock<std::mutex> lk(mu_);
    if (!cv_.wait_until(lk, deadline, [this] { return !q_.empty(); })) return false;
    *out = std::move(q_.front());
    q_.erase(q_.begin());
    return true;
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<T> q_;
};

std::unique_ptr<lsp::Server> start_server(const lsp::Params& p, int* port) {
  std::string err;
  auto s = lsp::NewServer(0, p, &err);
  if (!s) fail("NewServer: " + err);
  else *port = s->Port();
  return s;
}

std::unique_ptr<lsp::Client> start_client(int port, const lsp::Params& p) {
  std::string err;
  auto c = lsp::NewClient(lspnet::JoinHostPort("localhost", port), p, &err);
  if (!c) fail("NewClient: " + err);
  return c;
}

// ----------------------------------------------------------------------------
// lsp1_test.go: echo server, clients write (i + random) and expect the echo.
// ----------------------------------------------------------------------------
bool echo_test(int nclients, lsp::Params prm, int nmsgs, int max_sleep, int drop, int timeout_ms) {
  int port = 0;
  auto srv = start_server(prm, &port);
  if (!srv) return false;
  std::vector<std::unique_ptr<lsp::Client>> cli;
  for (int i = 0; i < nclients; ++i) {
    cli.push_back(start_client(port, prm));
    if (!cli.back()) return false;
  }
  lspnet::SetWriteDropPercent(drop);
  std::atomic<bool> exit_{false};
  std::thread server([&] {
    while (!exit_) {
      int id;
      std::string data;
      if (!srv->Read(&id, &data)) return;
      if (max_sleep > 0) sleep_ms(rnd(max_sleep));
      srv->Write(id, data);
    }
  });
  Chan<bool> done;
  std::vector<std::thread> ths;
  for (int c = 0; c < nclients; ++c) {
    ths.emplace_back([&, c] {
      lsp::Client* cl = cli[c].get();
      for (int i = 0; i < nmsgs && !exit_; ++i) {
        const int v = i + rnd(100);
        std::string err;
        if (!cl->Write(std::to_string(v), &err)) { fail("client write: " + err); done.put(false); return; }
        std::string got;
        if (!cl->Read(&got, &err)) { fail("client read: " + err); done.put(false); return; }
        if (got != std::to_string(v)) { fail("client got " + got + ", want " + std::to_string(v)); done.put(false); return; }
      }
      done.put(true);
    });
  }
  const auto deadline = steady_clock::now() + milliseconds(timeout_ms);
  bool ok = true;
  for (int c = 0; c < nclients && ok; ++c) {
    bool v;
    if (!done.get(&v, deadline)) { fail("timed out after " + std::to_string(timeout_ms) + " ms"); ok = false; }
    else if (!v) ok = false;
  }
  bail_if_failed(ok);
  exit_ = true;
  for (auto& t : ths) t.join();
  lspnet::ResetDropPercent();
  srv->Close();  // clients still ack; then the server thread's Read returns
  server.join();
  cli.clear();
  srv.reset();
  return true;
}

// ----------------------------------------------------------------------------
// Not in the reference: Params::Copies > 1.  Clients stream numbered messages
// to an echo server; every side must see each message exactly once and in
// order, and nothing more arrives after several epochs (of resends and
// heartbeats) -- a duplicate that slipped through would show up as an extra
// or out-of-order message.
// ----------------------------------------------------------------------------
bool dup_test(int copies, int drop) {
  lsp::Params prm = P(20, 100, 4);
  prm.Copies = copies;
  const int nclients = 3, nmsgs = 150;
  int port = 0;
  auto srv = start_server(prm, &port);
  if (!srv) return false;
  std::vector<std::unique_ptr<lsp::Client>> cli;
  for (int i = 0; i < nclients; ++i) {
    cli.push_back(start_client(port, prm));
    if (!cli.back()) return false;
  }
  lspnet::SetWriteDropPercent(drop);
  Chan<std::pair<int, std::string>> at_server, at_clients;
  std::thread server([&] {
    for (;;) {
      int id;
      std::string d;
      if (!srv->Read(&id, &d)) return;
      at_server.put({id, d});
      srv->Write(id, d);
    }
  });
  std::vector<std::thread> ths;
  for (int c = 0; c < nclients; ++c) {
    ths.emplace_back([&, c] {
      for (int i = 0; i < nmsgs; ++i) cli[c]->Write(std::to_string(c) + ":" + std::to_string(i));
      std::string d;
      while (cli[c]->Read(&d)) at_clients.put({c, d});
    });
  }
  auto check = [&](Chan<std::pair<int, std::string>>& ch, bool by_conn, const char* who) {
    std::map<int, int> next;  // sender -> next expected index
    const auto deadline = steady_clock::now() + seconds(20);
    for (int k = 0; k < nclients * nmsgs; ++k) {
      std::pair<int, std::string> e;
      if (!ch.get(&e, deadline)) { fail(std::string(who) + ": timed out"); return false; }
      const size_t colon = e.second.find(':');
      const int c = atoi(e.second.substr(0, colon).c_str()), i = atoi(e.second.substr(colon + 1).c_str());
      const int key = by_conn ? e.first : c;
      if (!by_conn && c != e.first) { fail(std::string(who) + ": client got another client's echo"); return false; }
      if (i != next[key]) {
        fail(std::string(who) + ": message " + e.second + " out of order or duplicated (want index " +
             std::to_string(next[key]) + ")");
        return false;
      }
      next[key]++;
    }
    return true;
  };
  bool ok = check(at_server, true, "server") && check(at_clients, false, "clients");
  if (ok) {
    // 6 epochs of resends / heartbeats: no message may be delivered again
    std::pair<int, std::string> e;
    if (at_server.get(&e, steady_clock::now() + milliseconds(600)) ||
        at_clients.get(&e, steady_clock::now() + milliseconds(10))) {
      fail("extra delivery after the stream: " + e.second);
      ok = false;
    }
  }
  bail_if_failed(ok);
  lspnet::ResetDropPercent();
  for (auto& c : cli) c->Close();
  for (auto& t : ths) t.join();
  srv->Close();
  server.join();
  return true;
}

// ----------------------------------------------------------------------------
// lsp2_test.go: window tests.
// ----------------------------------------------------------------------------
std::vector<std::string> rand_msgs(int n) {
  std::vector<std::string> v;
  for (int i = 0; i < n; ++i) v.push_back(std::to_string(rnd(1 << 30)));
  return v;
}

bool window_test(bool max_capacity, int nclients, int nmsgs, lsp::Params prm, int max_epochs) {
  const int W = prm.WindowSize;
  int port = 0;
  auto srv = start_server(prm, &port);
  if (!srv) return false;
  std::map<int, std::unique_ptr<lsp::Client>> cli;
  for (int i = 0; i < nclients; ++i) {
    auto c = start_client(port, prm);
    if (!c) return false;
    const int id = c->ConnID();
    cli[id] = std::move(c);
  }
  const auto server_msgs = rand_msgs(nmsgs), client_msgs = rand_msgs(nmsgs);
  std::mutex mu;
  std::map<int, std::vector<std::string>> srv_read, cli_read;  // by conn id
  Chan<bool> sdone, cdone;
  const auto deadline = steady_clock::now() + milliseconds(max_epochs * prm.EpochMillis);
  std::vector<std::thread> ths;
  auto wait = [&](Chan<bool>& ch, const char* who) {
    bool v;
    if (!ch.get(&v, deadline)) { fail(std::string("timed out waiting for ") + who); return false; }
    if (!v) { fail(std::string(who) + " failed"); return false; }
    return true;
  };
  auto stream_to_server = [&](lsp::Client* c, std::vector<std::string> msgs) {
    for (auto& m : msgs)
      if (!c->Write(m)) { cdone.put(false); return; }
    cdone.put(true);
  };
  auto stream_to_client = [&](int id, std::vector<std::string> msgs) {
    for (auto& m : msgs)
      if (!srv->Write(id, m)) { sdone.put(false); return; }
    sdone.put(true);
  };
  auto read_from_all_clients = [&](int total, int checkpoint) {
    for (int i = 0; i < total; ++i) {
      if (i == checkpoint) sdone.put(true);
      int id;
      std::string d;
      if (!srv->Read(&id, &d)) { sdone.put(false); return; }
      std::lock_guard<std::mutex> g(mu);
      srv_read[id].push_back(d);
    }
    sdone.put(true);
  };
  auto read_from_server = [&](int id, lsp::Client* c, int total, int checkpoint) {
    for (int i = 0; i < total; ++i) {
      if (i == checkpoint) cdone.put(true);
      std::string d;
      if (!c->Read(&d)) { cdone.put(false); return; }
      std::lock_guard<std::mutex> g(mu);
      cli_read[id].push_back(d);
    }
    cdone.put(true);
  };
  auto check = [&](std::map<int, std::vector<std::string>>& got, const std::vector<std::string>& want,
                   const char* who) {
    std::lock_guard<std::mutex> g(mu);
    for (auto& kv : cli) {
      auto& v = got[kv.first];
      if (v != want) {
        fail(std::string(who) + " of conn " + std::to_string(kv.first) + " read " + std::to_string(v.size()) +
             " msgs, want " + std::to_string(want.size()));
        return false;
      }
    }
    return true;
  };
  bool ok = true;
  if (max_capacity) {
    // (1) client -> server with the server unable to ack: only W arrive
    lspnet::SetServerWriteDropPercent(100);
    ths.emplace_back(read_from_all_clients, nclients * nmsgs, W * nclients);
    for (auto& kv : cli) ths.emplace_back(stream_to_server, kv.second.get(), client_msgs);
    for (int i = 0; i < nclients && ok; ++i) ok = wait(cdone, "clients");
    ok = ok && wait(sdone, "server");
    sleep_ms(50);
    ok = ok && check(srv_read, std::vector<std::string>(client_msgs.begin(), client_msgs.begin() + W), "server");
    lspnet::SetServerWriteDropPercent(0);
    ok = ok && wait(sdone, "server");
    sleep_ms(50);
    ok = ok && check(srv_read, client_msgs, "server");
    // (2) server -> client with the clients unable to ack
    lspnet::SetClientWriteDropPercent(100);
    for (auto& kv : cli) {
      ths.emplace_back(read_from_server, kv.first, kv.second.get(), nmsgs, W);
      ths.emplace_back(stream_to_client, kv.first, server_msgs);
    }
    for (int i = 0; i < nclients && ok; ++i) ok = wait(sdone, "server");
    for (int i = 0; i < nclients && ok; ++i) ok = wait(cdone, "clients");
    sleep_ms(50);
    ok = ok && check(cli_read, std::vector<std::string>(server_msgs.begin(), server_msgs.begin() + W), "client");
    lspnet::SetClientWriteDropPercent(0);
    for (int i = 0; i < nclients && ok; ++i) ok = wait(cdone, "clients");
    sleep_ms(50);
    ok = ok && check(cli_read, server_msgs, "client");
  } else {
    const int half = nmsgs / 2;
    // (1) client -> server: the first half is lost on the way, the second arrives first
    lspnet::SetClientWriteDropPercent(100);
    for (auto& kv : cli)
      ths.emplace_back(stream_to_server, kv.second.get(),
                       std::vector<std::string>(client_msgs.begin(), client_msgs.begin() + half));
    for (int i = 0; i < nclients && ok; ++i) ok = wait(cdone, "clients");
    lspnet::SetClientWriteDropPercent(0);
    for (auto& kv : cli)
      ths.emplace_back(stream_to_server, kv.second.get(),
                       std::vector<std::string>(client_msgs.begin() + half, client_msgs.end()));
    for (int i = 0; i < nclients && ok; ++i) ok = wait(cdone, "clients");
    ths.emplace_back(read_from_all_clients, nmsgs * nclients, 0);
    ok = ok && wait(sdone, "server");
    sleep_ms(50);
    ok = ok && wait(sdone, "server");
    sleep_ms(50);
    ok = ok && check(srv_read, client_msgs, "server");
    // (2) server -> clients, same
    lspnet::SetServerWriteDropPercent(100);
    for (auto& kv : cli)
      ths.emplace_back(stream_to_client, kv.first,
                       std::vector<std::string>(server_msgs.begin(), server_msgs.begin() + half));
    for (int i = 0; i < nclients && ok; ++i) ok = wait(sdone, "server");
    lspnet::SetServerWriteDropPercent(0);
    for (auto& kv : cli)
      ths.emplace_back(stream_to_client, kv.first, std::vector<std::string>(server_msgs.begin() + half, server_msgs.end()));
    for (int i = 0; i < nclients && ok; ++i) ok = wait(sdone, "server");
    for (auto& kv : cli) ths.emplace_back(read_from_server, kv.first, kv.second.get(), nmsgs, 0);
    for (int i = 0; i < nclients && ok; ++i) ok = wait(cdone, "clients");
    sleep_ms(50);
    for (int i = 0; i < nclients && ok; ++i) ok = wait(cdone, "clients");
    sleep_ms(50);
    ok = ok && check(cli_read, server_msgs, "client");
  }
  bail_if_failed(ok);
  lspnet::ResetDropPercent();
  for (auto& t : ths) t.join();
  cli.clear();
  srv.reset();
  return true;
}

// ----------------------------------------------------------------------------
// lsp3_test.go: close tests.  Clients send numMsgs values and expect echoes.
// ----------------------------------------------------------------------------
enum CloseMode { kSlowStart, kServerClose, kServerCloseConns, kClientClose };

bool close_test(CloseMode mode, int nclients, int max_epochs, lsp::Params prm) {
  const int nmsgs = 10, delay_epochs = 3;
  // the clients need the port before the (delayed) server exists: reserve one
  int port = 0;
  {
    auto probe = start_server(prm, &port);
    if (!probe) return false;
    probe->Close();
  }
  std::vector<std::unique_ptr<lsp::Client>> cli(nclients);
  std::unique_ptr<lsp::Server> srv;
  std::mutex srv_mu;
  std::condition_variable srv_cv;
  Chan<bool> sdone, cdone;
  std::atomic<bool> exit_{false};
  std::atomic<int> ready{0};
  std::thread server([&] {
    if (mode == kSlowStart) sleep_ms(delay_epochs * prm.EpochMillis);
    std::string err;
    auto s = lsp::NewServer(port, prm, &err);
    if (!s) { fail("server start: " + err); sdone.put(false); return; }
    lsp::Server* S = s.get();
    {
      std::lock_guard<std::mutex> g(srv_mu);
      srv = std::move(s);
    }
    srv_cv.notify_all();
    int dead = 0, echoed = 0;
    while (!exit_) {
      int id;
      std::string data;
      if (!S->Read(&id, &data)) {
        if (exit_) return;
        ++dead;
        if (mode == kClientClose && dead == nclients) { sdone.put(true); S->Close(); return; }
        continue;
      }
      if (!S->Write(id, data)) { fail("server write"); sdone.put(false); return; }
      if (++echoed == nclients * nmsgs) {
        if (mode == kServerClose) { S->Close(); sdone.put(true); return; }
        if (mode == kServerCloseConns) {
          while (ready < nclients) sleep_ms(1);
          for (auto& c : cli) S->CloseConn(c->ConnID());
          sdone.put(true);
          return;
        }
        if (mode != kClientClose) { sdone.put(true); S->CloseConn(id); return; }
      }
    }
  });
  std::vector<std::thread> ths;
  for (int i = 0; i < nclients; ++i) {
    ths.emplace_back([&, i] {
      std::string err;
      auto c = lsp::NewClient(lspnet::JoinHostPort("localhost", port), prm, &err);
      if (!c) { fail("client connect: " + err); cdone.put(false); return; }
      lsp::Client* C = c.get();
      cli[i] = std::move(c);
      ready++;
      for (int m = 0; m < nmsgs && !exit_; ++m) {
        const std::string tv = std::to_string(m * 100 + rnd(100));
        if (!C->Write(tv)) { fail("client write"); cdone.put(false); return; }
        std::string got;
        if (!C->Read(&got)) { fail("client saw server termination early"); cdone.put(false); return; }
        if (got != tv) { fail("client got " + got + " want " + tv); cdone.put(false); return; }
      }
      if (mode == kClientClose) {
        C->Close();
        cdone.put(true);
      } else if (mode == kServerCloseConns || mode == kServerClose) {
        std::string got;
        if (C->Read(&got)) { fail("client read unexpected data after server close"); cdone.put(false); return; }
        cdone.put(true);
      } else {
        C->Close();
        cdone.put(true);
      }
    });
  }
  const auto deadline = steady_clock::now() + milliseconds(max_epochs * prm.EpochMillis);
  bool ok = true;
  auto wait = [&](Chan<bool>& ch, const char* who) {
    bool v;
    if (!ch.get(&v, deadline)) { fail(std::string("timed out waiting for ") + who); return false; }
    return v;
  };
  if (mode == kClientClose) {
    ok = wait(sdone, "server");
    for (int i = 0; i < nclients && ok; ++i) ok = wait(cdone, "client");
  } else {
    for (int i = 0; i < nclients && ok; ++i) ok = wait(cdone, "client");
    ok = ok && wait(sdone, "server");
  }
  bail_if_failed(ok);
  exit_ = true;
  for (auto& t : ths) t.join();
  server.join();
  cli.clear();
  srv.reset();
  return true;
}

// ----------------------------------------------------------------------------
// lsp4_test.go: sync tests.  A master toggles the network (100% write drop)
// around client/server phases; Close calls are issued while the network is
// off and must complete once it is back.
// ----------------------------------------------------------------------------
enum SyncMode { kServerFastClose, kServerToClient, kClientToServer, kRoundTrip };

bool sync_test(SyncMode mode, int nclients, int nmsgs, lsp::Params prm, int max_epochs) {
  int port = 0;
  std::unique_ptr<lsp::Server> srv = start_server(prm, &port);
  if (!srv) return false;
  std::vector<std::vector<int>> data(nclients, std::vector<int>(nmsgs));
  for (auto& v : data)
    for (int& x : v) x = rnd(1 << 30);
  std::vector<std::unique_ptr<lsp::Client>> cli(nclients);
  std::map<int, int> client_of;  // conn id -> client index
  std::mutex map_mu;
  // master <-> server / clients; s2m/c2m carry 0 ok, 1 error.  One signal
  // channel per client: with a shared one, a fast client could take a signal
  // meant for a slower one (Go's unbuffered channel hands them out in turn)
  Chan<int> m2s, s2m, c2m;
  std::vector<Chan<int>> m2c(nclients);
  const auto deadline = steady_clock::now() + milliseconds(max_epochs * prm.EpochMillis);
  std::atomic<bool> exit_{false};
  lspnet::SetWriteDropPercent(0);
  auto await = [&](Chan<int>& ch) {
    int v;
    while (!exit_) {
      if (ch.get(&v, steady_clock::now() + milliseconds(50))) return true;
    }
    return false;
  };
  std::thread server([&] {
    s2m.put(0);
    if (mode != kServerToClient) {
      if (!await(m2s)) return;
      std::vector<int> rcvd(nclients, 0);
      for (int m = 0; m < nmsgs * nclients; ++m) {
        int id;
        std::string b;
        if (!srv->Read(&id, &b)) { fail("server read failed"); s2m.put(1); return; }
        std::lock_guard<std::mutex> g(map_mu);
        auto it = client_of.find(id);
        if (it == client_of.end()) { fail("message from unknown client"); s2m.put(1); return; }
        const int ci = it->second;
        if (rcvd[ci] >= nmsgs || std::to_string(data[ci][rcvd[ci]]) != b) {
          fail("server received unexpected element");
          s2m.put(1);
          return;
        }
        rcvd[ci]++;
      }
      s2m.put(0);
    }
    if (mode != kClientToServer) {
      if (!await(m2s)) return;
      std::vector<int> sent(nclients, 0);
      for (int n = 0; n < nmsgs * nclients;) {
        int ci;
        do ci = rnd(nclients);
        while (sent[ci] >= nmsgs);
        if (!srv->Write(cli[ci]->ConnID(), std::to_string(data[ci][sent[ci]]))) {
          fail("server write failed");
          s2m.put(1);
          return;
        }
        sent[ci]++;
        n++;
      }
      s2m.put(0);
    }
    if (!await(m2s)) return;
    srv->Close();
    s2m.put(0);
  });
  std::vector<std::thread> ths;
  for (int i = 0; i < nclients; ++i) {
    ths.emplace_back([&, i] {
      std::string err;
      auto c = lsp::NewClient(lspnet::JoinHostPort("localhost", port), prm, &err);
      if (!c) { fail("client connect: " + err); c2m.put(1); return; }
      lsp::Client* C = c.get();
      {
        std::lock_guard<std::mutex> g(map_mu);
        client_of[C->ConnID()] = i;
        cli[i] = std::move(c);
      }
      c2m.put(0);
      if (mode != kServerToClient) {
        if (!await(m2c[i])) return;
        for (int n = 0; n < nmsgs; ++n)
          if (!C->Write(std::to_string(data[i][n]), &err)) { fail("client write failed: " + err); c2m.put(1); return; }
        c2m.put(0);
      }
      if (mode != kClientToServer) {
        if (!await(m2c[i])) return;
        for (int n = 0; n < nmsgs; ++n) {
          std::string b;
          if (!C->Read(&b)) { fail("client read failed at #" + std::to_string(n)); c2m.put(1); return; }
          if (b != std::to_string(data[i][n])) { fail("client received unexpected element"); c2m.put(1); return; }
        }
        c2m.put(0);
      }
      if (!await(m2c[i])) return;
      C->Close();
      c2m.put(0);
    });
  }
  auto wait_server = [&] {
    int v;
    if (!s2m.get(&v, deadline)) { fail("timed out waiting for server"); return false; }
    return v == 0;
  };
  auto wait_clients = [&] {
    for (int i = 0; i < nclients; ++i) {
      int v;
      if (!c2m.get(&v, deadline)) { fail("timed out waiting for clients"); return false; }
      if (v) return false;
    }
    return true;
  };
  auto signal_clients = [&] {
    for (int i = 0; i < nclients; ++i) m2c[i].put(0);
  };
  bool net_off = false;
  auto toggle = [&] {
    net_off = !net_off;
    lspnet::SetWriteDropPercent(net_off ? 100 : 0);
    if (!net_off) sleep_ms(2 * prm.EpochMillis);  // lsp4_test.go:135-136
  };
  // lsp4_test.go:380-442 (master)
  bool ok = wait_server() && wait_clients();
  if (ok) toggle();  // network off
  if (ok && mode != kServerToClient) {
    signal_clients();
    ok = wait_clients();
  }
  if (ok && mode == kClientToServer) signal_clients();  // fast close of clients
  if (ok && mode != kServerToClient) {
    toggle();  // on
    if (mode == kClientToServer) ok = wait_clients();
    if (ok) toggle();  // off
    if (ok) {
      m2s.put(0);  // server reads
      ok = wait_server();
    }
  }
  if (ok && mode != kClientToServer) {
    m2s.put(0);  // server writes
    ok = wait_server();
  }
  if (ok && mode != kRoundTrip) m2s.put(0);  // fast close of the server
  if (ok && mode != kClientToServer) {
    toggle();  // on
    if (mode != kRoundTrip) ok = wait_server();
    if (ok) toggle();  // off
    if (ok) {
      signal_clients();  // client reads
      ok = wait_clients();
    }
    if (ok) {
      signal_clients();  // client closes
      ok = wait_clients();
    }
  }
  if (ok && mode == kRoundTrip) {  // final close by the server
    m2s.put(0);
    ok = wait_server();
  }
  bail_if_failed(ok);
  exit_ = true;
  lspnet::ResetDropPercent();
  for (auto& t : ths) t.join();
  server.join();
  cli.clear();
  srv.reset();
  return true;
}

// ----------------------------------------------------------------------------
// lsp5_test.go: variable-length payloads (Size field checks).
// ----------------------------------------------------------------------------
bool varlen_test(bool server_reads, int timeout_ms) {
  lsp::Params prm = P(5, 2000, 1);
  int port = 0;
  auto srv = start_server(prm, &port);
  if (!srv) return false;
  auto cli = start_client(port, prm);
  if (!cli) return false;
  const std::string data = std::to_string(rnd(1000) * 1000);
  auto send = [&] {
    if (server_reads) cli->Write(data);
    else srv->Write(cli->ConnID(), data);
  };
  Chan<std::string> got;
  std::thread reader([&] {
    for (;;) {
      std::string d;
      int id;
      const bool r = server_reads ? srv->Read(&id, &d) : cli->Read(&d);
      if (!r) return;
      got.put(d);
    }
  });
  bool ok = true;
  std::string d;
  send();  // normal
  if (!got.get(&d, steady_clock::now() + milliseconds(timeout_ms)) || d != data) { fail("normal message"); ok = false; }
  lspnet::SetMsgLengtheningPercent(100);  // longer payload than Size: truncated
  if (ok) send();
  if (ok && (!got.get(&d, steady_clock::now() + milliseconds(timeout_ms)) || d.size() != data.size())) {
    fail("long message not truncated");
    ok = false;
  }
  lspnet::SetMsgLengtheningPercent(0);
  lspnet::SetMsgShorteningPercent(100);  // shorter payload than Size: never delivered
  if (ok) send();
  if (ok && got.get(&d, steady_clock::now() + milliseconds(timeout_ms))) { fail("short message delivered: " + d); ok = false; }
  lspnet::SetMsgShorteningPercent(0);
  bail_if_failed(ok);
  if (server_reads) srv->Close();  // unblocks the reader
  else cli->Close();
  reader.join();
  cli.reset();
  srv.reset();
  return true;
}

const std::map<std::string, std::function<bool()>>& scenarios() {
  static const std::map<std::string, std::function<bool()>> m = {
      // not in the reference: first transmissions sent 3x (Params::Copies),
      // every message delivered exactly once, in order, both directions
      {"DuplicatesExactlyOnce", [] { return dup_test(3, 0); }},
      {"DuplicatesUnderDrop", [] { return dup_test(2, 15); }},
      // lsp1_test.go
      {"Basic1", [] { return echo_test(1, P(5, 2000, 1), 3, 0, 0, 2000); }},
      {"Basic2", [] { return echo_test(1, P(5, 2000, 1), 50, 0, 0, 2000); }},
      {"Basic3", [] { return echo_test(2, P(5, 2000, 1), 50, 0, 0, 2000); }},
      {"Basic4", [] { return echo_test(10, P(5, 2000, 2), 50, 0, 0, 2000); }},
      {"Basic5", [] { return echo_test(2, P(5, 2000, 2), 500, 0, 0, 2000); }},
      {"Basic6", [] { return echo_test(10, P(5, 2000, 20), 500, 0, 0, 15000); }},
      {"Basic7", [] { return echo_test(4, P(5, 2000, 2), 10, 100, 0, 15000); }},
      {"Basic8", [] { return echo_test(5, P(5, 2000, 10), 10, 100, 0, 15000); }},
      {"Basic9", [] { return echo_test(2, P(5, 2000, 10), 50, 100, 0, 15000); }},
      {"SendReceive1", [] { return echo_test(1, P(3, 5000, 1), 6, 0, 0, 5000); }},
      {"SendReceive2", [] { return echo_test(4, P(3, 5000, 1), 6, 0, 0, 5000); }},
      {"SendReceive3", [] { return echo_test(4, P(3, 10000, 1), 6, 100, 0, 10000); }},
      {"Robust1", [] { return echo_test(1, P(20, 50, 1), 10, 0, 20, 15000); }},
      {"Robust2", [] { return echo_test(3, P(20, 50, 1), 15, 0, 20, 15000); }},
      {"Robust3", [] { return echo_test(5, P(20, 50, 1), 10, 0, 20, 15000); }},
      {"Robust4", [] { return echo_test(1, P(20, 50, 2), 10, 0, 20, 15000); }},
      {"Robust5", [] { return echo_test(3, P(20, 50, 5), 15, 0, 20, 15000); }},
      {"Robust6", [] { return echo_test(5, P(20, 50, 10), 10, 0, 20, 15000); }},
      // lsp2_test.go
      {"Window1", [] { return window_test(true, 1, 10, P(3, 500, 5), 5); }},
      {"Window2", [] { return window_test(true, 5, 25, P(3, 500, 10), 5); }},
      {"Window3", [] { return window_test(true, 10, 25, P(3, 500, 10), 5); }},
      {"Window4", [] { return window_test(false, 1, 10, P(3, 1000, 20), 5); }},
      {"Window5", [] { return window_test(false, 5, 10, P(3, 1000, 20), 5); }},
      {"Window6", [] { return window_test(false, 10, 10, P(3, 1000, 20), 5); }},
      // lsp3_test.go
      {"ServerSlowStart1", [] { return close_test(kSlowStart, 1, 5, P(5, 500, 1)); }},
      {"ServerSlowStart2", [] { return close_test(kSlowStart, 3, 5, P(5, 500, 1)); }},
      {"ServerClose1", [] { return close_test(kServerClose, 1, 10, P(5, 500, 1)); }},
      {"ServerClose2", [] { return close_test(kServerClose, 3, 5, P(2, 500, 1)); }},
      {"ServerCloseConns1", [] { return close_test(kServerCloseConns, 1, 10, P(5, 500, 1)); }},
      {"ServerCloseConns2", [] { return close_test(kServerCloseConns, 3, 5, P(2, 500, 1)); }},
      {"ClientClose1", [] { return close_test(kClientClose, 2, 10, P(5, 500, 1)); }},
      {"ClientClose2", [] { return close_test(kClientClose, 3, 15, P(5, 500, 1)); }},
      // lsp4_test.go
      {"ServerFastClose1", [] { return sync_test(kServerFastClose, 1, 10, P(5, 500, 1), 12); }},
      {"ServerFastClose2", [] { return sync_test(kServerFastClose, 3, 10, P(5, 500, 1), 12); }},
      {"ServerFastClose3", [] { return sync_test(kServerFastClose, 5, 500, P(5, 2000, 1), 20); }},
      {"ServerToClient1", [] { return sync_test(kServerToClient, 1, 10, P(5, 500, 1), 12); }},
      {"ServerToClient2", [] { return sync_test(kServerToClient, 3, 10, P(5, 500, 1), 12); }},
      {"ServerToClient3", [] { return sync_test(kServerToClient, 5, 500, P(5, 2000, 1), 20); }},
      {"ClientToServer1", [] { return sync_test(kClientToServer, 1, 10, P(5, 500, 1), 12); }},
      {"ClientToServer2", [] { return sync_test(kClientToServer, 3, 10, P(5, 500, 1), 12); }},
      {"ClientToServer3", [] { return sync_test(kClientToServer, 5, 500, P(5, 2000, 1), 20); }},
      {"RoundTrip1", [] { return sync_test(kRoundTrip, 1, 10, P(5, 500, 1), 12); }},
      {"RoundTrip2", [] { return sync_test(kRoundTrip, 3, 10, P(5, 500, 1), 12); }},
      {"RoundTrip3", [] { return sync_test(kRoundTrip, 5, 500, P(5, 2000, 1), 20); }},
      // lsp5_test.go
      {"VariableLengthMsgServer", [] { return varlen_test(true, 2000); }},
      {"VariableLengthMsgClient", [] { return varlen_test(false, 2000); }},
  };
  return m;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc == 4 && std::string(argv[1]) == "--copies") {  // [--copies K] <scenario>
    g_copies = atoi(argv[2]);
    argv += 2;
    argc -= 2;
  }
  if (argc != 2) {
    fprintf(stderr, "usage: %s [--copies K] <scenario> | --list\n", argv[0]);
    return 2;
  }
  const std::string name = argv[1];
  if (name == "--list") {
    for (auto& kv : scenarios()) printf("%s\n", kv.first.c_str());
    return 0;
  }
  auto it = scenarios().find(name);
  if (it == scenarios().end()) {
    fprintf(stderr, "unknown scenario %s\n", name.c_str());
    return 2;
  }
  const auto t0 = steady_clock::now();
  const bool ok = it->second();
  const double s = duration<double>(steady_clock::now() - t0).count();
  printf("%s %s %.2fs\n", name.c_str(), ok ? "PASS" : "FAIL", s);
  return ok ? 0 : 1;
}
