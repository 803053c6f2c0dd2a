// p1server -- the bitcoin server: splits client requests into chunks,
// schedules them over GPU-backed miners and returns each client the min
// (hash, nonce) of its range (configs[4]).
//
// Reference: /root/reference/src/github.com/cmu440/bitcoin/server/server.go
// (job policy: scheduler.hpp).  Two transports, one scheduler:
//
//   p1server [opts] lsp <port>                    server.go:45-170 over LSP/UDP:
//       prints "Server listening on port P" (port 0 picks one, server.go:79);
//       miners connect with `p1miner lsp host:port` and send Join, clients with
//       `p1client host:port msg maxNonce` send a Request; every message is the
//       encoding/json bitcoin.Message in an LSP payload.  A lost miner's chunk
//       is re-queued, a lost client's request dropped.  --exit-after N: exit 0
//       after answering N requests (tests, benchmarks); otherwise runs forever.
//   p1server [opts] scan <msg> <lower> <upper>    one request over child-process
//       miners ("p1miner serve" on pipes); prints "Result <hash> <nonce>"
//   p1server [opts] serve                         JSON Requests on stdin -> JSON
//       Results on stdout, in request order, over child-process miners
//
// opts: --chunk C (nonces per miner job, default 2^32)
//   lsp:   --epoch-limit K --epoch-millis M --window W (lsp.Params; default
//          NewParams(): 5, 2000, 1).  P1LSP_* env vars inject loss (lspnet.hpp).
//   pipes: --miners N (default 1)  --devices d0,d1,.. (device of miner i =
//          devices[i % len]; default 0)  --miner-cmd "CMD" (shell command per
//          miner, "{dev}" -> its device; default <dir>/p1miner serve --device {dev})
#include <errno.h>
#include <fcntl.h>
#include <inttypes.h>
#include <poll.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include <iostream>
#include <map>
#include <string>
#include <vector>

#include "bitcoin.hpp"
#include "gojson.hpp"
#include "lsp.hpp"
#include "lspnet.hpp"
#include "scheduler.hpp"

namespace {

// ----------------------------------------------------------------------------
// LSP transport (server.go:83-168)
// ----------------------------------------------------------------------------
int run_lsp(int port, const lsp::Params& prm, uint64_t chunk, long exit_after) {
  std::string err;
  std::unique_ptr<lsp::Server> srv = lsp::NewServer(port, prm, &err);
  if (!srv) {
    printf("%s\n", err.c_str());
    return 1;
  }
  printf("Server listening on port %d\n", srv->Port());
  fflush(stdout);
  sched::Scheduler S(chunk);
  long answered = 0;
  for (;;) {
    int id = 0;
    std::string payload;
    if (!srv->Read(&id, &payload, &err)) {
      if (id == 0) return 1;  // server closed
      // a lost connection: a miner's chunk is re-queued, a client's request dropped
      if (S.IsMiner(id)) S.LoseMiner(id);
      else S.CancelClient(id);
    } else {
      // server.go:117 ignores Unmarshal's error and switches on whatever was
      // decoded: a type error (say a negative Lower) still yields the rest of
      // the message.  Unlike the reference, a payload that is not JSON at all
      // is dropped rather than read as a zero Message (a Join).
      bitcoin::Message m;
      if (bitcoin::UnmarshalStatus(payload, &m) != gojson::kSyntaxError) {
        switch (m.Type) {
          case bitcoin::Join: S.AddMiner(id); break;
          case bitcoin::Request: S.Submit(id, m.Data, m.Lower, m.Upper); break;
          case bitcoin::Result: S.Result(id, m.Hash, m.Nonce); break;
        }
      }
    }
    for (const sched::Assignment& a : S.Dispatch())
      if (!srv->Write(a.miner, bitcoin::Marshal(bitcoin::NewRequest(a.data, a.lo, a.hi)))) S.Unassign(a.miner);
    for (const sched::Done& d : S.TakeDone()) {
      srv->Write((int)d.client, bitcoin::Marshal(bitcoin::NewResult(d.hash, d.nonce)));  // client may be gone
      if (exit_after > 0 && ++answered >= exit_after) {
        srv->Close();  // blocks until the results are acknowledged
        return 0;
      }
    }
  }
}

// ----------------------------------------------------------------------------
// Child-process transport: each miner is "p1miner serve" on a pipe pair,
// speaking newline-delimited encoding/json bitcoin.Message.
// ----------------------------------------------------------------------------
struct Child {
  pid_t pid = -1;
  int in_fd = -1, out_fd = -1;
  std::string buf;
};

std::string dir_of_self() {
  char p[4096];
  ssize_t n = readlink("/proc/self/exe", p, sizeof p - 1);
  if (n <= 0) return ".";
  p[n] = 0;
  std::string s(p);
  size_t k = s.rfind('/');
  return k == std::string::npos ? "." : s.substr(0, k);
}

bool spawn(Child& m, const std::string& cmd) {
  int in_p[2], out_p[2];
  if (pipe(in_p) || pipe(out_p)) return false;
  pid_t pid = fork();
  if (pid < 0) return false;
  if (pid == 0) {
    dup2(in_p[0], 0);
    dup2(out_p[1], 1);
    close(in_p[0]); close(in_p[1]); close(out_p[0]); close(out_p[1]);
    execl("/bin/sh", "sh", "-c", cmd.c_str(), (char*)nullptr);
    _exit(127);
  }
  close(in_p[0]);
  close(out_p[1]);
  m.pid = pid;
  m.in_fd = in_p[1];
  m.out_fd = out_p[0];
  return true;
}

void reap(Child& m) {
  if (m.in_fd >= 0) close(m.in_fd);
  if (m.out_fd >= 0) close(m.out_fd);
  m.in_fd = m.out_fd = -1;
  if (m.pid > 0) {
    int st;
    if (waitpid(m.pid, &st, WNOHANG) == 0) {
      kill(m.pid, SIGTERM);
      waitpid(m.pid, &st, 0);
    }
  }
  m.pid = -1;
}

bool write_all(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    ssize_t n = write(fd, s.data() + off, s.size() - off);
    if (n < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    off += (size_t)n;
  }
  return true;
}

class PipeServer {
 public:
  PipeServer(int nminers, std::vector<int> devs, uint64_t chunk, std::string cmd) : S_(chunk) {
    if (cmd.empty()) cmd = dir_of_self() + "/p1miner serve --device {dev}";
    for (int i = 0; i < nminers; ++i) {
      Child m;
      std::string c = cmd;
      const int dev = devs.empty() ? 0 : devs[i % devs.size()];
      for (size_t k; (k = c.find("{dev}")) != std::string::npos;) c.replace(k, 5, std::to_string(dev));
      if (!spawn(m, c)) { fprintf(stderr, "p1server: cannot start miner %d\n", i); continue; }
      kids_[i] = m;
      S_.AddMiner(i);
    }
  }
  ~PipeServer() {
    for (auto& kv : kids_) reap(kv.second);
  }
  size_t miners() const { return S_.Miners(); }
  uint64_t submit(const std::string& data, uint64_t lo, uint64_t hi) { return S_.Submit(0, data, lo, hi); }

  // Run until every request is answered; done(id, hash, nonce) in completion
  // order.  false if every miner is lost with work left.
  template <typename F>
  bool run(F done) {
    for (;;) {
      for (const sched::Done& d : S_.TakeDone()) done(d.req, d.hash, d.nonce);
      if (S_.Idle()) return true;
      for (const sched::Assignment& a : S_.Dispatch()) {
        const std::string line = bitcoin::Marshal(bitcoin::NewRequest(a.data, a.lo, a.hi)) + "\n";
        if (!write_all(kids_[a.miner].in_fd, line)) lose(a.miner);
      }
      if (S_.Starved()) return false;
      std::vector<pollfd> pf;
      std::vector<int> who;
      for (auto& kv : kids_) {
        pf.push_back({kv.second.out_fd, POLLIN, 0});
        who.push_back(kv.first);
      }
      if (poll(pf.data(), pf.size(), -1) < 0) {
        if (errno == EINTR) continue;
        return false;
      }
      for (size_t k = 0; k < pf.size(); ++k) {
        if (!(pf[k].revents & (POLLIN | POLLHUP | POLLERR))) continue;
        Child& m = kids_[who[k]];
        char tmp[4096];
        ssize_t n = read(m.out_fd, tmp, sizeof tmp);
        if (n <= 0) {  // miner lost: its chunk is re-queued (server.go:86-115 intent)
          lose(who[k]);
          continue;
        }
        m.buf.append(tmp, (size_t)n);
        size_t nl;
        while ((nl = m.buf.find('\n')) != std::string::npos) {
          std::string line = m.buf.substr(0, nl);
          m.buf.erase(0, nl + 1);
          bitcoin::Message res;
          if (bitcoin::Unmarshal(line, &res) && res.Type == bitcoin::Result) S_.Result(who[k], res.Hash, res.Nonce);
        }
      }
    }
  }

 private:
  void lose(int miner) {
    S_.LoseMiner(miner);
    auto it = kids_.find(miner);
    if (it != kids_.end()) {
      reap(it->second);
      kids_.erase(it);
    }
  }

  sched::Scheduler S_;
  std::map<int, Child> kids_;
};

int usage() {
  fprintf(stderr,
          "usage: p1server [--chunk C] [--epoch-limit K] [--epoch-millis M] [--window W] [--copies K] [--exit-after N] "
          "lsp <port>\n"
          "       p1server [--chunk C] [--miners N] [--devices d0,d1,..] [--miner-cmd CMD] "
          "scan <msg> <lower> <upper> | serve\n");
  return 2;
}

bool parse_u64(const char* s, uint64_t* v) {
  char* end = nullptr;
  if (!s || !*s || *s == '-') return false;
  errno = 0;
  unsigned long long r = strtoull(s, &end, 10);
  if (errno || *end) return false;
  *v = r;
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  signal(SIGPIPE, SIG_IGN);
  lspnet::ConfigureFromEnv();
  int nminers = 1;
  std::vector<int> devs;
  uint64_t chunk = 1ull << 32;
  std::string cmd;
  lsp::Params prm = lsp::NewParams();
  prm.Copies = lsp::DefaultAppCopies;
  long exit_after = 0;
  int i = 1;
  for (; i < argc; ++i) {
    if (!strcmp(argv[i], "--miners") && i + 1 < argc) nminers = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--devices") && i + 1 < argc) {
      std::string s = argv[++i];
      for (size_t a = 0; a < s.size();) {
        size_t b = s.find(',', a);
        if (b == std::string::npos) b = s.size();
        devs.push_back(atoi(s.substr(a, b - a).c_str()));
        a = b + 1;
      }
    } else if (!strcmp(argv[i], "--chunk") && i + 1 < argc) {
      if (!parse_u64(argv[++i], &chunk) || chunk == 0) return usage();
    } else if (!strcmp(argv[i], "--miner-cmd") && i + 1 < argc) cmd = argv[++i];
    else if (!strcmp(argv[i], "--epoch-limit") && i + 1 < argc) prm.EpochLimit = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--epoch-millis") && i + 1 < argc) prm.EpochMillis = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--window") && i + 1 < argc) prm.WindowSize = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--copies") && i + 1 < argc) prm.Copies = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--exit-after") && i + 1 < argc) exit_after = atol(argv[++i]);
    else break;
  }
  if (i >= argc || nminers < 1 || prm.EpochLimit < 1 || prm.EpochMillis < 1 || prm.WindowSize < 1) return usage();
  const std::string mode = argv[i];
  if (mode == "lsp" && i + 2 == argc) {
    char* end = nullptr;
    const long port = strtol(argv[i + 1], &end, 10);
    if (*end || port < 0 || port > 65535) {
      printf("Port must be a number: %s\n", argv[i + 1]);  // server.go:68-72
      return 1;
    }
    return run_lsp((int)port, prm, chunk, exit_after);
  }
  if (mode != "scan" && mode != "serve") return usage();
  PipeServer srv(nminers, devs, chunk, cmd);
  if (srv.miners() == 0) { fprintf(stderr, "p1server: no miner started\n"); return 1; }
  if (mode == "scan" && i + 4 == argc) {
    uint64_t lo, hi;
    if (!parse_u64(argv[i + 2], &lo) || !parse_u64(argv[i + 3], &hi)) return usage();
    srv.submit(argv[i + 1], lo, hi);
    bool ok = srv.run([](uint64_t, uint64_t h, uint64_t n) { printf("Result %" PRIu64 " %" PRIu64 "\n", h, n); });
    if (!ok) { printf("Disconnected\n"); return 1; }  // client.go:64-66
    return 0;
  }
  if (mode == "serve" && i + 1 == argc) {
    std::string line;
    while (std::getline(std::cin, line)) {
      bitcoin::Message req;
      if (bitcoin::UnmarshalStatus(line, &req) == gojson::kSyntaxError || req.Type != bitcoin::Request) continue;
      srv.submit(req.Data, req.Lower, req.Upper);
    }
    // stdio has no per-client connection (the reference answers each client
    // on its own LSP connection), so results are printed in request order
    std::map<uint64_t, std::pair<uint64_t, uint64_t>> ready;
    uint64_t next = 1;
    bool ok = srv.run([&](uint64_t id, uint64_t h, uint64_t n) {
      ready[id] = {h, n};
      for (auto it = ready.find(next); it != ready.end(); it = ready.find(next)) {
        printf("%s\n", bitcoin::Marshal(bitcoin::NewResult(it->second.first, it->second.second)).c_str());
        ready.erase(it);
        ++next;
      }
      fflush(stdout);
    });
    return ok ? 0 : 1;
  }
  return usage();
}
