// lsp.cpp -- see lsp.hpp.  Protocol: p1.pdf 2.1 (connection, data/ack,
// sliding window, epochs); reference implementation (for the API and the
// parts it has) /root/reference/src/github.com/cmu440/lsp/{client,server}_impl.go
// and common.go (sorter + window).
#include "lsp.hpp"

#include <errno.h>
#include <poll.h>
#include <sys/eventfd.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "lsp_message.hpp"
#include "lspnet.hpp"

namespace lsp {

std::string Params::String() const {
  return "[EpochLimit: " + std::to_string(EpochLimit) + ", EpochMillis: " + std::to_string(EpochMillis) +
         ", WindowSize: " + std::to_string(WindowSize) + "]";
}

Params NewParams() { return Params(); }

namespace {

using Clock = std::chrono::steady_clock;
constexpr size_t kMaxDatagram = 65536;

bool set_err(std::string* err, const std::string& what) {
  if (err) *err = what;
  return false;
}

// ----------------------------------------------------------------------------
// One side of one connection: the send window and the in-order receiver
// (common.go's slidingWindow and sorter, as plain state driven by the loop).
// ----------------------------------------------------------------------------
struct Peer {
  int64_t conn_id = 0;
  lspnet::UDPAddr addr;
  struct Out {
    int64_t seq;
    std::string payload;
    bool sent = false, acked = false;
  };
  int64_t next_seq = 1;   // sequence number of the next Write
  int64_t base = 1;       // oldest un-acked sequence number
  std::deque<Out> out;    // seq base .. next_seq-1
  int64_t expect = 1;     // next sequence number to deliver in order
  std::map<int64_t, std::string> early;  // received ahead of `expect`
  size_t early_bytes = 0;                 // payload bytes held in `early`
  bool got_data = false;  // any data message received (heartbeat choice)
  int idle = 0;           // epochs since anything arrived from the peer
  bool lost = false;
  int copies = 1;         // datagrams per first transmission (Params::Copies)
};

using SendFn = std::function<void(const Message&)>;
using DeliverFn = std::function<void(std::string&&)>;

// The first transmission of a message goes out p.copies times (the receiver
// acks every copy and keeps only new sequence numbers, so a duplicate is
// harmless); epoch resends go out once, as in the reference.
void send_data(Peer& p, Peer::Out& o, const SendFn& send) {
  const Message m = NewData(p.conn_id, o.seq, (int64_t)o.payload.size(), o.payload);
  for (int i = o.sent ? 1 : p.copies; i > 0; --i) send(m);
  o.sent = true;
}

// Send every message that the window now admits: seq in [base, base + W).
void pump(Peer& p, int window, const SendFn& send) {
  for (Peer::Out& o : p.out) {
    if (o.seq >= p.base + window) break;
    if (!o.sent) send_data(p, o, send);
  }
}

void queue_write(Peer& p, std::string&& payload, int window, const SendFn& send) {
  p.out.push_back({p.next_seq++, std::move(payload)});
  pump(p, window, send);
}

void on_ack(Peer& p, int64_t seq, int window, const SendFn& send) {
  if (seq < p.base || seq >= p.next_seq) return;  // heartbeat (0), stale or bogus
  p.out[(size_t)(seq - p.base)].acked = true;
  while (!p.out.empty() && p.out.front().acked) {
    p.out.pop_front();
    p.base++;
  }
  pump(p, window, send);
}

// A data message (Size already checked).  Every copy is acked -- the first
// ack may have been lost; only new sequence numbers are kept, and delivery
// is strictly in order (p1.pdf 2.1.2).
// A correct sender never has a message at or beyond expect + ITS WindowSize
// in flight (its window starts at its oldest un-acked message, which is at or
// below our `expect`).  The peer's WindowSize is its own Params, not ours
// (crunner/srunner take -wsize each), so the bound is a fixed generous cap
// and never our own window: anything kMaxEarly or more ahead is dropped
// un-acked, as if lost (the sender resends it an epoch later), which bounds
// `early` instead of letting a faulty peer grow it without limit.
// The same holds for bytes: a correct sender's early messages are at most a
// window of them, so more than kMaxEarlyBytes of payload held ahead of
// `expect` is a faulty peer, and a new early message beyond it is dropped
// un-acked too (64 KB datagrams x 2^16 sequence numbers would be 4 GB).
// A server also caps the early bytes of ALL its connections together
// (kMaxEarlyBytesAll, `pool`): a connection costs one unauthenticated Connect,
// so a per-connection cap alone would let many of them hold 64 MB each.
// And per source host (kMaxEarlyBytesHost, `host_pool`): without it one
// peer opening 4 connections from 4 ports fills the whole pool, and every
// other connection's out-of-order Data is then dropped until those time out
// (ADVICE r05).  A host's connections together hold what one may.
constexpr int64_t kMaxEarly = 1 << 16;
constexpr size_t kMaxEarlyBytes = 64u << 20;
constexpr size_t kMaxEarlyBytesAll = 256u << 20;
constexpr size_t kMaxEarlyBytesHost = kMaxEarlyBytes;
void on_data(Peer& p, Message& m, int window, const SendFn& send, const DeliverFn& deliver, size_t* pool = nullptr,
             size_t* host_pool = nullptr) {
  (void)window;
  if (m.SeqNum >= p.expect + kMaxEarly) return;
  if (m.SeqNum > p.expect && !p.early.count(m.SeqNum) &&
      (p.early_bytes + m.Payload.size() > kMaxEarlyBytes ||
       (pool && *pool + m.Payload.size() > kMaxEarlyBytesAll) ||
       (host_pool && *host_pool + m.Payload.size() > kMaxEarlyBytesHost)))
    return;
  send(NewAck(p.conn_id, m.SeqNum));
  p.got_data = true;
  if (m.SeqNum < p.expect) return;
  std::string payload(m.Payload.begin(), m.Payload.end());
  if (m.SeqNum > p.expect) {
    const size_t n = payload.size();
    if (p.early.emplace(m.SeqNum, std::move(payload)).second) {
      p.early_bytes += n;
      if (pool) *pool += n;
      if (host_pool) *host_pool += n;
    }
    return;
  }
  deliver(std::move(payload));
  p.expect++;
  for (auto it = p.early.find(p.expect); it != p.early.end(); it = p.early.find(p.expect)) {
    p.early_bytes -= it->second.size();
    if (pool) *pool -= it->second.size();
    if (host_pool) *host_pool -= it->second.size();
    deliver(std::move(it->second));
    p.early.erase(it);
    p.expect++;
  }
}

// Size check of p1.pdf 2.1.4: shorter payload -> as if dropped; longer -> truncated.
bool size_ok(Message& m) {
  if (m.Size < 0 || (int64_t)m.Payload.size() < m.Size) return false;
  if ((int64_t)m.Payload.size() > m.Size) m.Payload.resize((size_t)m.Size);
  return true;
}

// One epoch for a connection (p1.pdf 2.1.3): count idleness, heartbeat,
// resend the un-acked messages of the window.  Marks the peer lost after
// EpochLimit epochs of silence.
void on_epoch(Peer& p, const Params& prm, const SendFn& send) {
  if (++p.idle >= prm.EpochLimit) {
    p.lost = true;
    return;
  }
  send(NewAck(p.conn_id, p.got_data ? p.expect - 1 : 0));
  for (Peer::Out& o : p.out) {
    if (o.seq >= p.base + prm.WindowSize) break;
    if (o.sent && !o.acked) send_data(p, o, send);
  }
}

// ----------------------------------------------------------------------------
// Event loop shared by client and server: poll(socket, eventfd) with the next
// epoch as the timeout.  Callbacks run under the endpoint's mutex.
// ----------------------------------------------------------------------------
class Loop {
 public:
  Loop(lspnet::UDPConn* conn, std::mutex* mu, int epoch_ms,
       std::function<void(Message&, const lspnet::UDPAddr&)> on_msg, std::function<void()> on_tick)
      : conn_(conn), mu_(mu), epoch_(std::chrono::milliseconds(epoch_ms > 0 ? epoch_ms : 1)),
        on_msg_(std::move(on_msg)), on_tick_(std::move(on_tick)) {
    wake_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  }
  ~Loop() {
    Stop();
    if (wake_ >= 0) close(wake_);
  }
  void Start() { th_ = std::thread([this] { Run(); }); }
  void Stop() {
    if (!th_.joinable()) return;
    stop_ = true;
    uint64_t one = 1;
    (void)!write(wake_, &one, sizeof one);
    if (th_.get_id() == std::this_thread::get_id()) th_.detach();
    else th_.join();
  }

 private:
  void Run() {
    std::vector<uint8_t> buf(kMaxDatagram);
    auto next = Clock::now() + epoch_;
    while (!stop_) {
      const auto now = Clock::now();
      int timeout = 0;
      if (next > now) timeout = (int)std::chrono::ceil<std::chrono::milliseconds>(next - now).count();
      pollfd pf[2] = {{conn_->fd(), POLLIN, 0}, {wake_, POLLIN, 0}};
      int rc = poll(pf, 2, timeout);
      if (stop_) break;
      // POLLERR without POLLIN: a pending ICMP error (e.g. port unreachable
      // after the server died) on the connected client socket.  recvfrom
      // consumes it (ECONNREFUSED below); left alone, poll would return at
      // once on every iteration and spin until the next epoch's send.
      if (rc > 0 && (pf[0].revents & (POLLIN | POLLERR))) {
        for (;;) {  // drain every queued datagram
          lspnet::UDPAddr from;
          ssize_t n = conn_->ReadFromUDP(buf.data(), buf.size(), &from);
          if (n == lspnet::UDPConn::kDropped) continue;
          if (n < 0) {
            if (errno == EAGAIN || errno == EWOULDBLOCK) break;
            if (errno == ECONNREFUSED || errno == EINTR) continue;  // an earlier send bounced: consumed
            break;
          }
          Message m;
          if (!Unmarshal(std::string((const char*)buf.data(), (size_t)n), &m)) continue;
          std::lock_guard<std::mutex> g(*mu_);
          on_msg_(m, from);
        }
      }
      if (Clock::now() >= next) {
        {
          std::lock_guard<std::mutex> g(*mu_);
          on_tick_();
        }
        next += epoch_;
        if (next < Clock::now()) next = Clock::now() + epoch_;  // never fire a burst of stale epochs
      }
    }
  }

  lspnet::UDPConn* conn_;
  std::mutex* mu_;
  std::chrono::milliseconds epoch_;
  std::function<void(Message&, const lspnet::UDPAddr&)> on_msg_;
  std::function<void()> on_tick_;
  int wake_ = -1;
  std::thread th_;
  std::atomic<bool> stop_{false};
};

// ----------------------------------------------------------------------------
// Client
// ----------------------------------------------------------------------------
class ClientImpl : public Client {
 public:
  ClientImpl(std::unique_ptr<lspnet::UDPConn> conn, const Params& prm)
      : conn_(std::move(conn)), prm_(prm) {
    send_ = [this](const Message& m) { conn_->Write(Marshal(m)); };
    loop_.reset(new Loop(
        conn_.get(), &mu_, prm_.EpochMillis, [this](Message& m, const lspnet::UDPAddr&) { on_msg(m); },
        [this] { on_tick(); }));
  }
  ~ClientImpl() override { shutdown(); }

  // client_impl.go:40-80 (NewClient): Connect, resent every epoch, until the
  // server's Ack(id, 0); give up after EpochLimit epochs.
  bool Connect(std::string* err) {
    {
      std::lock_guard<std::mutex> g(mu_);
      p_.copies = prm_.Copies > 1 ? prm_.Copies : 1;  // Data only
      // one Connect per attempt by default: a reference server opens a
      // connection per Connect datagram (Params::ConnectCopies)
      const int cc = prm_.ConnectCopies > 1 ? prm_.ConnectCopies : 1;
      for (int i = 0; i < cc; ++i) send_(NewConnect());
    }
    loop_->Start();
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] { return connected_ || lost_; });
    if (!connected_) {
      lk.unlock();
      shutdown();
      return set_err(err, "lsp: no answer to the connection request after " + std::to_string(prm_.EpochLimit) +
                              " epochs");
    }
    return true;
  }

  int ConnID() const override { return (int)p_.conn_id; }

  bool Read(std::string* payload, std::string* err) override {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] { return !inbox_.empty() || lost_ || closed_; });
    if (!inbox_.empty()) {
      *payload = std::move(inbox_.front());
      inbox_.pop_front();
      return true;
    }
    return set_err(err, lost_ ? "lsp: connection lost" : "lsp: connection closed");
  }

  bool Write(const std::string& payload, std::string* err) override {
    std::lock_guard<std::mutex> g(mu_);
    if (lost_) return set_err(err, "lsp: connection lost");
    if (closed_) return set_err(err, "lsp: connection closed");
    queue_write(p_, std::string(payload), prm_.WindowSize, send_);
    return true;
  }

  bool Close(std::string* err) override {
    bool lost;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] { return p_.out.empty() || lost_; });
      lost = lost_;
      closed_ = true;
    }
    cv_.notify_all();
    shutdown();
    return lost ? set_err(err, "lsp: connection lost before all messages were acknowledged") : true;
  }

 private:
  void on_msg(Message& m) {
    if (!connected_) {
      // client_impl.go:195-199: the Ack of the connection request carries the id
      if (m.Type == MsgAck && m.SeqNum == 0) {
        connected_ = true;
        p_.conn_id = m.ConnID;
        p_.idle = 0;
        cv_.notify_all();
      }
      return;
    }
    if (m.ConnID != p_.conn_id || lost_) return;
    if (m.Type == MsgData && !size_ok(m)) return;
    p_.idle = 0;
    if (m.Type == MsgAck) {
      on_ack(p_, m.SeqNum, prm_.WindowSize, send_);
      if (p_.out.empty()) cv_.notify_all();  // Close may be waiting
    } else if (m.Type == MsgData) {
      on_data(p_, m, prm_.WindowSize, send_, [this](std::string&& s) { inbox_.push_back(std::move(s)); });
      cv_.notify_all();
    }
  }

  void on_tick() {
    if (lost_) return;
    if (!connected_) {
      if (++connect_epochs_ >= prm_.EpochLimit) {
        lost_ = true;
        cv_.notify_all();
        return;
      }
      send_(NewConnect());
      return;
    }
    on_epoch(p_, prm_, send_);
    if (p_.lost) {
      lost_ = true;
      cv_.notify_all();
    }
  }

  void shutdown() {
    loop_->Stop();
    std::lock_guard<std::mutex> g(mu_);
    closed_ = true;
    cv_.notify_all();
  }

  std::unique_ptr<lspnet::UDPConn> conn_;
  Params prm_;
  std::mutex mu_;
  std::condition_variable cv_;
  SendFn send_;
  Peer p_;
  std::deque<std::string> inbox_;
  bool connected_ = false, lost_ = false, closed_ = false;
  int connect_epochs_ = 0;
  std::unique_ptr<Loop> loop_;  // last: stopped first
};

// ----------------------------------------------------------------------------
// Server
// ----------------------------------------------------------------------------
class ServerImpl : public Server {
 public:
  ServerImpl(std::unique_ptr<lspnet::UDPConn> conn, const Params& prm) : conn_(std::move(conn)), prm_(prm) {
    loop_.reset(new Loop(
        conn_.get(), &mu_, prm_.EpochMillis, [this](Message& m, const lspnet::UDPAddr& a) { on_msg(m, a); },
        [this] { on_tick(); }));
    loop_->Start();
  }
  ~ServerImpl() override { shutdown(); }

  int Port() const override { return conn_->LocalPort(); }

  bool Read(int* connID, std::string* payload, std::string* err) override {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] { return !inbox_.empty() || closed_; });
    if (inbox_.empty()) {
      *connID = 0;
      return set_err(err, "lsp: server closed");
    }
    Event e = std::move(inbox_.front());
    inbox_.pop_front();
    *connID = (int)e.conn;
    if (e.lost) return set_err(err, "lsp: connection " + std::to_string(e.conn) + " lost");
    *payload = std::move(e.payload);
    return true;
  }

  bool Write(int connID, const std::string& payload, std::string* err) override {
    std::lock_guard<std::mutex> g(mu_);
    auto it = conns_.find(connID);
    if (it == conns_.end() || it->second.p.lost || it->second.closing)
      return set_err(err, "lsp: no connection " + std::to_string(connID));
    Conn& c = it->second;
    queue_write(c.p, std::string(payload), prm_.WindowSize, sender(c));
    return true;
  }

  bool CloseConn(int connID, std::string* err) override {
    std::lock_guard<std::mutex> g(mu_);
    auto it = conns_.find(connID);
    if (it == conns_.end() || it->second.closing) return set_err(err, "lsp: no connection " + std::to_string(connID));
    it->second.closing = true;
    // server_api.go:19-21: no data from an explicitly closed connection is returned
    for (auto e = inbox_.begin(); e != inbox_.end();) e = (e->conn == connID) ? inbox_.erase(e) : e + 1;
    reap();
    return true;
  }

  bool Close(std::string* err) override {
    bool any_lost;
    {
      std::unique_lock<std::mutex> lk(mu_);
      closing_all_ = true;
      for (auto& kv : conns_) kv.second.closing = true;
      reap();
      cv_.wait(lk, [this] { return conns_.empty(); });
      any_lost = lost_while_closing_;
    }
    shutdown();
    return any_lost ? set_err(err, "lsp: a connection was lost before its messages were acknowledged") : true;
  }

 private:
  struct Conn {
    Peer p;
    std::string host;      // source address without the port (kMaxEarlyBytesHost)
    bool closing = false;  // CloseConn / Close: drain pending, deliver nothing
  };

  static std::string host_of(const lspnet::UDPAddr& a) {
    std::string s = a.String();
    const size_t colon = s.rfind(':');
    return colon == std::string::npos ? s : s.substr(0, colon);
  }
  struct Event {
    int64_t conn;
    std::string payload;
    bool lost;
  };

  SendFn sender(Conn& c) {
    const lspnet::UDPAddr a = c.p.addr;
    return [this, a](const Message& m) { conn_->WriteToUDP(Marshal(m), a); };
  }

  void on_msg(Message& m, const lspnet::UDPAddr& from) {
    if (closed_) return;
    if (m.Type == MsgConnect) {
      // duplicate requests from an address with a live connection get the
      // same id again (p1.pdf 2.1.3); ids are sequential from 1
      auto a = by_addr_.find(from);
      int64_t id;
      if (a != by_addr_.end() && conns_.count(a->second)) {
        id = a->second;
        conns_[id].p.idle = 0;
      } else {
        if (closing_all_) return;
        id = next_id_++;
        Conn c;
        c.p.conn_id = id;
        c.p.addr = from;
        c.host = host_of(from);
        c.p.copies = prm_.Copies > 1 ? prm_.Copies : 1;
        conns_.emplace(id, std::move(c));
        by_addr_[from] = id;
        // a new connection's Ack goes out `copies` times (first transmission)
        for (int i = 1; i < conns_[id].p.copies; ++i) conn_->WriteToUDP(Marshal(NewAck(id, 0)), from);
      }
      conn_->WriteToUDP(Marshal(NewAck(id, 0)), from);
      return;
    }
    auto it = conns_.find(m.ConnID);
    if (it == conns_.end()) return;
    Conn& c = it->second;
    // Only the connection's own address speaks for it.  The reference looks
    // the connection up by ConnID alone (server_impl.go:198-204), so any
    // datagram naming a live id and a plausible SeqNum could inject a
    // message or ack one the client never had delivered; a correct client
    // always sends from the socket it connected with.
    if (!(c.p.addr == from)) return;
    if (m.Type == MsgData && !size_ok(m)) return;
    c.p.idle = 0;
    const SendFn send = sender(c);
    if (m.Type == MsgAck) {
      on_ack(c.p, m.SeqNum, prm_.WindowSize, send);
      if (c.closing) reap();
    } else if (m.Type == MsgData) {
      const bool hide = c.closing;
      const int64_t id = c.p.conn_id;
      on_data(
          c.p, m, prm_.WindowSize, send,
          [this, hide, id](std::string&& s) {
            if (!hide) inbox_.push_back({id, std::move(s), false});
          },
          &early_all_, &early_by_host_[c.host]);
      cv_.notify_all();
    }
  }

  void on_tick() {
    for (auto& kv : conns_) on_epoch(kv.second.p, prm_, sender(kv.second));
    reap();
  }

  // Remove lost connections (reporting those the application did not close)
  // and closing ones whose pending messages are all acked.
  void reap() {
    bool changed = false;
    for (auto it = conns_.begin(); it != conns_.end();) {
      Conn& c = it->second;
      const bool done = c.p.lost || (c.closing && c.p.out.empty());
      if (!done) {
        ++it;
        continue;
      }
      if (c.p.lost && !c.closing) inbox_.push_back({c.p.conn_id, std::string(), true});
      if (c.p.lost && closing_all_ && !c.p.out.empty()) lost_while_closing_ = true;
      auto a = by_addr_.find(c.p.addr);
      if (a != by_addr_.end() && a->second == c.p.conn_id) by_addr_.erase(a);
      early_all_ -= c.p.early_bytes;  // its held-back data leaves with it
      auto h = early_by_host_.find(c.host);
      if (h != early_by_host_.end() && (h->second -= c.p.early_bytes) == 0) early_by_host_.erase(h);
      it = conns_.erase(it);
      changed = true;
    }
    if (changed) cv_.notify_all();
  }

  void shutdown() {
    loop_->Stop();
    std::lock_guard<std::mutex> g(mu_);
    closed_ = true;
    cv_.notify_all();
  }

  std::unique_ptr<lspnet::UDPConn> conn_;
  Params prm_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<int64_t, Conn> conns_;
  std::map<lspnet::UDPAddr, int64_t> by_addr_;
  std::deque<Event> inbox_;
  int64_t next_id_ = 1;
  size_t early_all_ = 0;  // early bytes held by all connections (kMaxEarlyBytesAll)
  std::map<std::string, size_t> early_by_host_;  // early bytes per source host (kMaxEarlyBytesHost)
  bool closing_all_ = false, lost_while_closing_ = false, closed_ = false;
  std::unique_ptr<Loop> loop_;  // last: stopped first
};

}  // namespace

std::unique_ptr<Client> NewClient(const std::string& hostport, const Params& params, std::string* err) {
  lspnet::UDPAddr addr;
  if (!lspnet::ResolveUDPAddr(hostport, &addr, err)) return nullptr;
  std::unique_ptr<lspnet::UDPConn> conn = lspnet::UDPConn::DialUDP(addr, err);
  if (!conn) return nullptr;
  std::unique_ptr<ClientImpl> c(new ClientImpl(std::move(conn), params));
  if (!c->Connect(err)) return nullptr;
  return c;
}

std::unique_ptr<Server> NewServer(int port, const Params& params, std::string* err) {
  lspnet::UDPAddr addr;
  if (!lspnet::ResolveUDPAddr(lspnet::JoinHostPort("localhost", port), &addr, err)) return nullptr;
  std::unique_ptr<lspnet::UDPConn> conn = lspnet::UDPConn::ListenUDP(addr, err);
  if (!conn) return nullptr;
  return std::unique_ptr<Server>(new ServerImpl(std::move(conn), params));
}

}  // namespace lsp
