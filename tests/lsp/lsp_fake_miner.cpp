// lsp_fake_miner -- TEST DOUBLE for the LSP server's CPU tests: the miner
// loop of miner.go:13-73 over this repository's LSP, answering every request
// with the oracle (oracle/libp1oracle.so, the CPU checker) instead of the GPU.
//
//   lsp_fake_miner <host:port> [--epoch-limit K] [--epoch-millis M] [--window W] [--copies K] [--connect-copies K]
// FAKE_DIE_AFTER=n: after answering n requests, read the next one and exit
// without answering or closing (a miner the server must declare lost).
// FAKE_LOG=path: append "lower upper" of every request received (tests check
// what the server handed out).
// P1LSP_* env vars inject loss (lspnet.hpp).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <memory>
#include <string>

#include "../../p1_amd/host/bitcoin.hpp"
#include "../../p1_amd/host/lsp.hpp"
#include "../../p1_amd/host/lspnet.hpp"

extern "C" int p1o_scan(const uint8_t* msg, size_t len, uint64_t lower, uint64_t upper, uint64_t* out_hash,
                        uint64_t* out_nonce);

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  lspnet::ConfigureFromEnv();
  lsp::Params prm = lsp::NewParams();
  prm.Copies = lsp::DefaultAppCopies;  // like p1miner
  for (int i = 2; i < argc; ++i) {
    if (!strcmp(argv[i], "--epoch-limit") && i + 1 < argc) prm.EpochLimit = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--epoch-millis") && i + 1 < argc) prm.EpochMillis = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--window") && i + 1 < argc) prm.WindowSize = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--copies") && i + 1 < argc) prm.Copies = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--connect-copies") && i + 1 < argc) prm.ConnectCopies = atoi(argv[++i]);
    else return 2;
  }
  const char* die = getenv("FAKE_DIE_AFTER");
  const long die_after = die && *die ? atol(die) : -1;
  const char* logp = getenv("FAKE_LOG");
  std::string err;
  std::unique_ptr<lsp::Client> cli = lsp::NewClient(argv[1], prm, &err);
  if (!cli) {
    printf("Failed to join with server: %s\n", err.c_str());
    return 1;
  }
  cli->Write(bitcoin::Marshal(bitcoin::NewJoin()));
  long answered = 0;
  for (;;) {
    std::string buf;
    if (!cli->Read(&buf)) break;
    if (answered == die_after) _exit(3);  // vanish: no answer, no Close
    bitcoin::Message req;
    bitcoin::Unmarshal(buf, &req);  // miner.go:54-55: the error is ignored
    if (logp && *logp) {
      if (FILE* f = fopen(logp, "a")) {
        fprintf(f, "%llu %llu\n", (unsigned long long)req.Lower, (unsigned long long)req.Upper);
        fclose(f);
      }
    }
    uint64_t h = UINT64_MAX, n = 0;
    if (req.Lower <= req.Upper) p1o_scan((const uint8_t*)req.Data.data(), req.Data.size(), req.Lower, req.Upper, &h, &n);
    if (!cli->Write(bitcoin::Marshal(bitcoin::NewResult(h, n)))) break;
    ++answered;
  }
  cli->Close();
  return 0;
}
