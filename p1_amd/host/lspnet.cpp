// lspnet.cpp -- see lspnet.hpp.
#include "lspnet.hpp"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <random>

#include "lsp_message.hpp"

namespace lspnet {
namespace {

std::atomic<int> g_client_read{0}, g_client_write{0}, g_server_read{0}, g_server_write{0};
std::atomic<int> g_shorten{0}, g_lengthen{0};

void set(std::atomic<int>& a, int p) {
  if (0 <= p && p <= 100) a.store(p);
}

bool sometimes(int percent) {  // conn.go:131-133
  if (percent <= 0) return false;
  if (percent >= 100) return true;
  thread_local std::mt19937 rng(std::random_device{}());
  return (int)(rng() % 100u) < percent;
}

int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  return atoi(v);
}

}  // namespace

void SetClientReadDropPercent(int p) { set(g_client_read, p); }
void SetClientWriteDropPercent(int p) { set(g_client_write, p); }
void SetServerReadDropPercent(int p) { set(g_server_read, p); }
void SetServerWriteDropPercent(int p) { set(g_server_write, p); }
void SetReadDropPercent(int p) {
  SetClientReadDropPercent(p);
  SetServerReadDropPercent(p);
}
void SetWriteDropPercent(int p) {
  SetClientWriteDropPercent(p);
  SetServerWriteDropPercent(p);
}
void SetMsgShorteningPercent(int p) { set(g_shorten, p); }
void SetMsgLengtheningPercent(int p) { set(g_lengthen, p); }
void ResetDropPercent() {
  SetReadDropPercent(0);
  SetWriteDropPercent(0);
}

void ConfigureFromEnv() {
  int v;
  if ((v = env_int("P1LSP_READ_DROP", -1)) >= 0) SetReadDropPercent(v);
  if ((v = env_int("P1LSP_WRITE_DROP", -1)) >= 0) SetWriteDropPercent(v);
  if ((v = env_int("P1LSP_CLIENT_READ_DROP", -1)) >= 0) SetClientReadDropPercent(v);
  if ((v = env_int("P1LSP_CLIENT_WRITE_DROP", -1)) >= 0) SetClientWriteDropPercent(v);
  if ((v = env_int("P1LSP_SERVER_READ_DROP", -1)) >= 0) SetServerReadDropPercent(v);
  if ((v = env_int("P1LSP_SERVER_WRITE_DROP", -1)) >= 0) SetServerWriteDropPercent(v);
  if ((v = env_int("P1LSP_SHORTEN", -1)) >= 0) SetMsgShorteningPercent(v);
  if ((v = env_int("P1LSP_LENGTHEN", -1)) >= 0) SetMsgLengtheningPercent(v);
}

std::string UDPAddr::String() const {
  char host[INET6_ADDRSTRLEN] = "?";
  int port = 0;
  if (ss.ss_family == AF_INET) {
    const sockaddr_in* a = (const sockaddr_in*)&ss;
    inet_ntop(AF_INET, &a->sin_addr, host, sizeof host);
    port = ntohs(a->sin_port);
    return std::string(host) + ":" + std::to_string(port);
  }
  if (ss.ss_family == AF_INET6) {
    const sockaddr_in6* a = (const sockaddr_in6*)&ss;
    inet_ntop(AF_INET6, &a->sin6_addr, host, sizeof host);
    port = ntohs(a->sin6_port);
    return "[" + std::string(host) + "]:" + std::to_string(port);
  }
  return "?";
}

bool UDPAddr::operator==(const UDPAddr& o) const { return len == o.len && memcmp(&ss, &o.ss, len) == 0; }

bool UDPAddr::operator<(const UDPAddr& o) const {
  if (len != o.len) return len < o.len;
  return memcmp(&ss, &o.ss, len) < 0;
}

std::string JoinHostPort(const std::string& host, int port) {
  if (host.find(':') != std::string::npos) return "[" + host + "]:" + std::to_string(port);
  return host + ":" + std::to_string(port);
}

bool ResolveUDPAddr(const std::string& hostport, UDPAddr* out, std::string* err) {
  std::string host, port;
  if (!hostport.empty() && hostport[0] == '[') {
    size_t e = hostport.find("]:");
    if (e == std::string::npos) { if (err) *err = "missing port in address " + hostport; return false; }
    host = hostport.substr(1, e - 1);
    port = hostport.substr(e + 2);
  } else {
    size_t c = hostport.rfind(':');
    if (c == std::string::npos) { if (err) *err = "missing port in address " + hostport; return false; }
    host = hostport.substr(0, c);
    port = hostport.substr(c + 1);
  }
  if (host.empty()) host = "127.0.0.1";
  if (host == "localhost") host = "127.0.0.1";  // the container hostname may not resolve; localhost is IPv4 here
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_DGRAM;
  int rc = getaddrinfo(host.c_str(), port.c_str(), &hints, &res);
  if (rc != 0 || !res) {
    if (err) *err = "resolve " + hostport + ": " + gai_strerror(rc);
    return false;
  }
  memcpy(&out->ss, res->ai_addr, res->ai_addrlen);
  out->len = (socklen_t)res->ai_addrlen;
  freeaddrinfo(res);
  return true;
}

UDPConn::~UDPConn() { Close(); }

static int make_socket(int family, std::string* err) {
  int fd = socket(family, SOCK_DGRAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0 && err) *err = std::string("socket: ") + strerror(errno);
  if (fd >= 0) {
    int sz = 4 << 20;  // room for bursts of datagrams (many clients, wide windows)
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof sz);
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof sz);
  }
  return fd;
}

std::unique_ptr<UDPConn> UDPConn::ListenUDP(const UDPAddr& laddr, std::string* err) {
  int fd = make_socket(laddr.ss.ss_family, err);
  if (fd < 0) return nullptr;
  if (bind(fd, (const sockaddr*)&laddr.ss, laddr.len) != 0) {
    if (err) *err = "listen " + laddr.String() + ": " + strerror(errno);
    ::close(fd);
    return nullptr;
  }
  return std::unique_ptr<UDPConn>(new UDPConn(fd, true));
}

std::unique_ptr<UDPConn> UDPConn::DialUDP(const UDPAddr& raddr, std::string* err) {
  int fd = make_socket(raddr.ss.ss_family, err);
  if (fd < 0) return nullptr;
  if (connect(fd, (const sockaddr*)&raddr.ss, raddr.len) != 0) {
    if (err) *err = "dial " + raddr.String() + ": " + strerror(errno);
    ::close(fd);
    return nullptr;
  }
  return std::unique_ptr<UDPConn>(new UDPConn(fd, false));
}

int UDPConn::LocalPort() const {
  sockaddr_storage ss{};
  socklen_t len = sizeof ss;
  if (getsockname(fd_, (sockaddr*)&ss, &len) != 0) return -1;
  if (ss.ss_family == AF_INET) return ntohs(((sockaddr_in*)&ss)->sin_port);
  if (ss.ss_family == AF_INET6) return ntohs(((sockaddr_in6*)&ss)->sin6_port);
  return -1;
}

ssize_t UDPConn::ReadFromUDP(uint8_t* buf, size_t cap, UDPAddr* from) {
  sockaddr_storage ss{};
  socklen_t len = sizeof ss;
  ssize_t n = recvfrom(fd_, buf, cap, 0, (sockaddr*)&ss, &len);
  if (n < 0) return -1;
  // conn.go:52-70: a read the knob selects is discarded
  if (sometimes(server_ ? g_server_read.load() : g_client_read.load())) return kDropped;
  if (from) {
    memcpy(&from->ss, &ss, len);
    from->len = len;
  }
  return n;
}

ssize_t UDPConn::write_impl(const std::string& datagram, const UDPAddr* to) {
  // conn.go:99-104: drop, but make it look like it was successful
  if (sometimes(server_ ? g_server_write.load() : g_client_write.load())) return (ssize_t)datagram.size();
  const std::string* out = &datagram;
  std::string mangled;
  const int sh = g_shorten.load(), ln = g_lengthen.load();
  if (sh > 0 || ln > 0) {
    // conn.go:106-138: a Data message may leave with a shorter or longer
    // payload than its Size field says (the receiver must drop / truncate)
    lsp::Message m;
    if (lsp::Unmarshal(datagram, &m) && m.Type == lsp::MsgData) {
      const bool shorten = sometimes(sh);
      const bool lengthen = !shorten && sometimes(ln);
      if (shorten) m.Payload.resize(m.Payload.size() / 2);
      if (lengthen) m.Payload.insert(m.Payload.end(), {2, 3, 4});
      if (shorten || lengthen) {
        mangled = lsp::Marshal(m);
        out = &mangled;
      }
    }
  }
  ssize_t n = to ? sendto(fd_, out->data(), out->size(), 0, (const sockaddr*)&to->ss, to->len)
                 : send(fd_, out->data(), out->size(), 0);
  // a full socket buffer or an unreachable peer is a lost datagram to LSP
  return n < 0 ? (ssize_t)datagram.size() : n;
}

ssize_t UDPConn::WriteToUDP(const std::string& datagram, const UDPAddr& to) { return write_impl(datagram, &to); }

ssize_t UDPConn::Write(const std::string& datagram) { return write_impl(datagram, nullptr); }

void UDPConn::Close() {
  if (fd_ >= 0) ::close(fd_);
  fd_ = -1;
}

}  // namespace lspnet
