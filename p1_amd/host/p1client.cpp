// p1client -- the bitcoin client (client.go:13-66) over this repository's
// LSP: sends one Request [0, maxNonce] for <message> to the server and prints
// "Result <hash> <nonce>", or "Disconnected" if the connection is lost.
//
//   p1client <host:port> <message> <maxNonce> [--epoch-limit K]
//            [--epoch-millis M] [--window W] [--copies K] [--connect-copies K]
// Reference: /root/reference/src/github.com/cmu440/bitcoin/client/client.go
// P1LSP_* env vars inject loss (lspnet.hpp).
#include <errno.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <memory>
#include <string>

#include "bitcoin.hpp"
#include "lsp.hpp"
#include "lspnet.hpp"

int main(int argc, char** argv) {
  if (argc < 4) {
    printf("Usage: ./%s <hostport> <message> <maxNonce>", argv[0]);  // client.go:15-17
    return 2;
  }
  lspnet::ConfigureFromEnv();
  lsp::Params prm = lsp::NewParams();
  prm.Copies = lsp::DefaultAppCopies;
  for (int i = 4; i < argc; ++i) {
    if (!strcmp(argv[i], "--epoch-limit") && i + 1 < argc) prm.EpochLimit = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--epoch-millis") && i + 1 < argc) prm.EpochMillis = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--window") && i + 1 < argc) prm.WindowSize = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--copies") && i + 1 < argc) prm.Copies = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--connect-copies") && i + 1 < argc) prm.ConnectCopies = atoi(argv[++i]);
    else return 2;
  }
  const std::string hostport = argv[1], message = argv[2];
  char* end = nullptr;
  errno = 0;
  const unsigned long long max_nonce = strtoull(argv[3], &end, 10);
  if (errno || *end || argv[3][0] == '-' || !argv[3][0]) {
    printf("%s is not a number.\n", argv[3]);  // client.go:21-25
    return 1;
  }
  std::string err;
  std::unique_ptr<lsp::Client> cli = lsp::NewClient(hostport, prm, &err);
  if (!cli) {
    printf("Failed to connect to server: %s\n", err.c_str());  // client.go:27-31
    return 1;
  }
  std::string buf;
  if (!cli->Write(bitcoin::Marshal(bitcoin::NewRequest(message, 0, max_nonce))) || !cli->Read(&buf)) {
    printf("Disconnected\n");  // client.go:41-51, 63-66
    return 1;
  }
  bitcoin::Message res;
  bitcoin::Unmarshal(buf, &res);  // client.go:52-53 ignores the error
  printf("Result %" PRIu64 " %" PRIu64 "\n", res.Hash, res.Nonce);  // client.go:58-61
  fflush(stdout);
  cli->Close();  // client.go:33 (defer client.Close())
  return 0;
}
