// p1miner -- the miner's Request -> Result loop (miner.go:49-67), GPU-backed
// through libp1hip.so, over LSP (the reference's transport) or stdio.
// Requests/results are encoding/json bitcoin.Message bytes (miner.go:55,66).
//
//   p1miner lsp <host:port> [--device N] [--chunk C] [--epoch-limit K]
//           [--epoch-millis M] [--window W] [--copies K] [--connect-copies K]
//                                        miner.go:13-73: connect, send Join,
//                                        then Read -> scan -> Write until the
//                                        connection is lost.  The scan runs on
//                                        this thread while the LSP event loop
//                                        keeps heartbeating, so a long GPU job
//                                        never trips the epoch limit.
//
//   p1miner scan <msg> <lower> <upper>   prints "Result <hash> <nonce>"
//                                        (the client's output, client.go:59-61)
//   p1miner hash <msg> <nonce>           prints bitcoin.Hash(msg, nonce)
//   p1miner serve [--device N] [--chunk C]
//                                        one JSON Message per stdin line; every
//                                        line is answered with one JSON Result
//                                        line (miner.go:49-67 scans whatever it
//                                        decoded, as Go's Unmarshal leaves it)
//   p1miner json                         re-marshals stdin JSON lines (no GPU;
//                                        wire-format tests): "ERROR" for a
//                                        syntax error, "TYPEERROR\t" before
//                                        Go's partial decode on a type error
//   p1miner lsp-json                     re-marshals stdin lsp.Message JSON lines
//                                        (lsp/message.go; no GPU)
//   p1miner lsp-wrap <connID> <seq>      each stdin bitcoin.Message JSON line ->
//                                        the LSP Data datagram that carries it
//                                        (miner.go:66 client.Write), seq counting up
//   p1miner lsp-unwrap                   LSP Data datagram lines -> the bitcoin
//                                        message in their payload (miner.go:50-55)
#include <errno.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <iostream>
#include <memory>
#include <string>

#include "../../include/p1hip.h"
#include "bitcoin.hpp"
#include "gojson.hpp"
#include "lsp.hpp"
#include "lsp_message.hpp"
#include "lspnet.hpp"

static int usage() {
  fprintf(stderr,
          "usage: p1miner scan <msg> <lower> <upper> | hash <msg> <nonce> | "
          "serve [--device N] [--chunk C] | lsp <host:port> [--device N] [--chunk C] [--epoch-limit K] "
          "[--epoch-millis M] [--window W] [--copies K] [--connect-copies K] | json | lsp-json | lsp-wrap <connID> <seq> | lsp-unwrap\n");
  return 2;
}

static bool parse_u64(const char* s, uint64_t* v) {
  char* end = nullptr;
  if (!s || !*s || *s == '-') return false;
  errno = 0;
  unsigned long long r = strtoull(s, &end, 10);
  if (errno || *end) return false;
  *v = r;
  return true;
}

// miner.go:13-31 (joinWithServer) + miner.go:33-73 (main loop)
static int run_lsp(int argc, char** argv) {
  const std::string hostport = argv[2];
  int dev = -1;
  uint64_t chunk = miner::kDefaultChunk;
  lsp::Params prm = lsp::NewParams();
  prm.Copies = lsp::DefaultAppCopies;
  for (int i = 3; i < argc; ++i) {
    if (!strcmp(argv[i], "--device") && i + 1 < argc) dev = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--chunk") && i + 1 < argc) { if (!parse_u64(argv[++i], &chunk)) return usage(); }
    else if (!strcmp(argv[i], "--epoch-limit") && i + 1 < argc) prm.EpochLimit = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--epoch-millis") && i + 1 < argc) prm.EpochMillis = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--window") && i + 1 < argc) prm.WindowSize = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--copies") && i + 1 < argc) prm.Copies = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--connect-copies") && i + 1 < argc) prm.ConnectCopies = atoi(argv[++i]);
    else return usage();
  }
  // open the GPU before joining, so the first request does not pay for it
  int rc = dev >= 0 ? p1hip_init_devices(&dev, 1) : p1hip_init(0, nullptr);
  if (rc != P1HIP_OK) { fprintf(stderr, "p1hip init: %s\n", p1hip_last_error()); return 1; }
  std::string err;
  std::unique_ptr<lsp::Client> cli = lsp::NewClient(hostport, prm, &err);
  if (!cli) {
    printf("Failed to join with server: %s\n", err.c_str());
    return 1;
  }
  if (!cli->Write(bitcoin::Marshal(bitcoin::NewJoin()), &err)) {
    cli->Close();
    printf("Failed to join with server: %s\n", err.c_str());
    return 1;
  }
  for (;;) {
    std::string buf;
    if (!cli->Read(&buf)) break;
    bitcoin::Message req;
    bitcoin::Unmarshal(buf, &req);  // miner.go:54-55: a fresh Message, the error ignored (partial decode kept)
    const bitcoin::Message res = miner::HandleRequest(req, chunk);
    if (!cli->Write(bitcoin::Marshal(res))) break;
  }
  cli->Close();  // miner.go:47 (defer miner.Close())
  p1hip_shutdown();
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) return usage();
  const std::string cmd = argv[1];
  lspnet::ConfigureFromEnv();
  try {
    if (cmd == "lsp" && argc >= 3) return run_lsp(argc, argv);
    if (cmd == "scan" && argc == 5) {
      uint64_t lo, hi, h, n;
      if (!parse_u64(argv[3], &lo) || !parse_u64(argv[4], &hi)) return usage();
      miner::ScanChunked(argv[2], lo, hi, miner::kDefaultChunk, &h, &n);
      printf("Result %" PRIu64 " %" PRIu64 "\n", h, n);
      return 0;
    }
    if (cmd == "hash" && argc == 4) {
      uint64_t n;
      if (!parse_u64(argv[3], &n)) return usage();
      printf("%" PRIu64 "\n", bitcoin::Hash(argv[2], n));
      return 0;
    }
    if (cmd == "json") {
      std::string line;
      while (std::getline(std::cin, line)) {
        bitcoin::Message m;
        const int st = bitcoin::UnmarshalStatus(line, &m);
        if (st == gojson::kSyntaxError) { printf("ERROR\n"); continue; }
        // fwrite, not %s: a decoded string may hold NUL bytes
        const std::string o = (st == gojson::kTypeError ? "TYPEERROR\t" : "") + bitcoin::Marshal(m) + "\t" + m.String() + "\n";
        fwrite(o.data(), 1, o.size(), stdout);
      }
      return 0;
    }
    if (cmd == "lsp-json") {
      std::string line;
      while (std::getline(std::cin, line)) {
        lsp::Message m;
        const int st = lsp::UnmarshalStatus(line, &m);
        if (st == gojson::kSyntaxError) { printf("ERROR\n"); continue; }
        // fwrite, not %s: a decoded string may hold NUL bytes
        const std::string o = (st == gojson::kTypeError ? "TYPEERROR\t" : "") + lsp::Marshal(m) + "\t" + m.String() + "\n";
        fwrite(o.data(), 1, o.size(), stdout);
      }
      return 0;
    }
    if (cmd == "lsp-wrap" && argc == 4) {
      char* end = nullptr;
      const long long conn = strtoll(argv[2], &end, 10);
      if (*end) return usage();
      long long seq = strtoll(argv[3], &end, 10);
      if (*end) return usage();
      std::string line;
      while (std::getline(std::cin, line)) {
        bitcoin::Message m;
        if (!bitcoin::Unmarshal(line, &m)) { printf("ERROR\n"); continue; }
        const std::string payload = bitcoin::Marshal(m);
        printf("%s\n", lsp::Marshal(lsp::NewData(conn, seq++, (int64_t)payload.size(), payload)).c_str());
      }
      return 0;
    }
    if (cmd == "lsp-unwrap") {
      std::string line;
      while (std::getline(std::cin, line)) {
        lsp::Message d;
        bitcoin::Message m;
        if (!lsp::Unmarshal(line, &d) || d.Type != lsp::MsgData ||
            !bitcoin::Unmarshal(std::string(d.Payload.begin(), d.Payload.end()), &m)) {
          printf("ERROR\n");
          continue;
        }
        printf("%s\n", bitcoin::Marshal(m).c_str());
      }
      return 0;
    }
    if (cmd == "serve") {
      int dev = -1;
      uint64_t chunk = miner::kDefaultChunk;
      for (int i = 2; i < argc; ++i) {
        if (!strcmp(argv[i], "--device") && i + 1 < argc) dev = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--chunk") && i + 1 < argc) { if (!parse_u64(argv[++i], &chunk)) return usage(); }
        else return usage();
      }
      int rc = dev >= 0 ? p1hip_init_devices(&dev, 1) : p1hip_init(0, nullptr);
      if (rc != P1HIP_OK) { fprintf(stderr, "p1hip init: %s\n", p1hip_last_error()); return 1; }
      std::string line;
      while (std::getline(std::cin, line)) {
        // miner.go:54-55 decodes into a fresh Message and ignores the error,
        // then scans [Lower, Upper] whatever the Type: a line with a type
        // error scans what Go's partial decode holds, a line that is not JSON
        // the one-nonce request ("", [0, 0]); every line is answered, so a
        // server never waits on a miner that stays silent.
        bitcoin::Message req;
        bitcoin::Unmarshal(line, &req);
        bitcoin::Message res = miner::HandleRequest(req, chunk);
        printf("%s\n", bitcoin::Marshal(res).c_str());
        fflush(stdout);
      }
      p1hip_shutdown();
      return 0;
    }
  } catch (const bitcoin::HipError& e) {
    fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  return usage();
}
