// lspnet.hpp -- UDP datagram layer under the LSP transport, with the fault
// injection knobs the reference's tests (and configs[4]'s "5% drop") use.
//
// Reference (paths relative to /root/reference/src/github.com/cmu440):
//   lspnet/net.go:24-67     ResolveUDPAddr / ListenUDP / DialUDP / JoinHostPort:
//                           a connection knows whether a server or a client
//                           made it (the drop knobs are per side)
//   lspnet/conn.go:37-154   reads and writes through the knobs: a dropped
//                           write "looks successful"; a Data message may be
//                           shortened or lengthened on the way out
//   lspnet/staff.go:18-99   Set{Client,Server}{Read,Write}DropPercent,
//                           SetMsgShortening/LengtheningPercent, Reset
// The knobs are process-global (as in the reference); command-line tools
// additionally read them from the environment (ConfigureFromEnv), so a test
// can inject loss into separate server and miner processes.
#pragma once
#include <netinet/in.h>
#include <stddef.h>
#include <stdint.h>
#include <sys/socket.h>
#include <sys/types.h>

#include <memory>
#include <string>

namespace lspnet {

// staff.go:18-99 (percentages 0..100; out-of-range values are ignored)
void SetReadDropPercent(int p);
void SetWriteDropPercent(int p);
void SetClientReadDropPercent(int p);
void SetClientWriteDropPercent(int p);
void SetServerReadDropPercent(int p);
void SetServerWriteDropPercent(int p);
void SetMsgShorteningPercent(int p);
void SetMsgLengtheningPercent(int p);
void ResetDropPercent();  // read and write drop back to 0 (staff.go:94-97)

// P1LSP_READ_DROP, P1LSP_WRITE_DROP, P1LSP_CLIENT_READ_DROP,
// P1LSP_CLIENT_WRITE_DROP, P1LSP_SERVER_READ_DROP, P1LSP_SERVER_WRITE_DROP,
// P1LSP_SHORTEN, P1LSP_LENGTHEN (integers, percent).
void ConfigureFromEnv();

struct UDPAddr {
  sockaddr_storage ss{};
  socklen_t len = 0;
  std::string String() const;  // "host:port"
  bool operator==(const UDPAddr& o) const;
  bool operator<(const UDPAddr& o) const;
};

// "host:port" (IPv4 or IPv6 literal, or a name such as localhost) -> address.
bool ResolveUDPAddr(const std::string& hostport, UDPAddr* out, std::string* err);
std::string JoinHostPort(const std::string& host, int port);

// One UDP socket.  Reads return one datagram; a read the knobs drop returns
// kDropped (the caller treats it as nothing received).  Writes the knobs drop
// report success without sending.  Non-blocking: callers poll fd().
class UDPConn {
 public:
  static constexpr ssize_t kDropped = -2;
  ~UDPConn();
  // server side: bind to laddr (port 0 = ephemeral)
  static std::unique_ptr<UDPConn> ListenUDP(const UDPAddr& laddr, std::string* err);
  // client side: a socket connected to raddr
  static std::unique_ptr<UDPConn> DialUDP(const UDPAddr& raddr, std::string* err);

  ssize_t ReadFromUDP(uint8_t* buf, size_t cap, UDPAddr* from);
  ssize_t WriteToUDP(const std::string& datagram, const UDPAddr& to);
  ssize_t Write(const std::string& datagram);  // to the dialled peer
  int LocalPort() const;
  int fd() const { return fd_; }
  bool is_server() const { return server_; }
  void Close();

 private:
  UDPConn(int fd, bool server) : fd_(fd), server_(server) {}
  ssize_t write_impl(const std::string& datagram, const UDPAddr* to);
  int fd_;
  bool server_;
};

}  // namespace lspnet
