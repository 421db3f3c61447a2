// Core of dalle_amd._kvstore: record store, wire protocol, TCP server and a blocking client, with no
// Python dependency. kvstore.cpp wraps it for Python (pybind11); kvstore_stress.cpp drives it from
// many threads under ThreadSanitizer / AddressSanitizer+UBSan (tests/test_kvstore_sanitizers_cpu.py),
// the race-detection tier of SURVEY §5.2.
//
// Records: key -> { subkey -> (value bytes, expiration time, owner) }.
//   * STORE keeps the record with the later expiration (DHT semantics) and rejects a write to a
//     subkey owned by a different owner while the record is alive (owner-signed subkeys, D20).
//   * GET returns only unexpired subkeys; expired ones are dropped lazily.
//   * WAIT blocks server-side (condition variable) until a key has >= N live subkeys, a timeout,
//     or server shutdown: the primitive behind barriers / matchmaking of the collaborative optimizer.
// Wire format: u32 frame length, u8 opcode, then fields; strings/bytes are u32 length + payload,
// times are f64 (seconds since the epoch, the clock of get_dht_time()).
#pragma once

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

namespace dalle_kv {

enum Op : uint8_t { OP_STORE = 1, OP_GET = 2, OP_DELETE = 3, OP_KEYS = 4, OP_PING = 5, OP_WAIT = 6 };

inline double now_s() {
  using namespace std::chrono;
  return duration_cast<duration<double>>(system_clock::now().time_since_epoch()).count();
}

struct Buf {
  std::string d;
  void u8(uint8_t v) { d.push_back((char)v); }
  void u32(uint32_t v) { d.append((const char*)&v, 4); }
  void f64(double v) { d.append((const char*)&v, 8); }
  void str(const std::string& s) { u32((uint32_t)s.size()); d.append(s); }
};

struct Reader {
  const std::string& d;
  size_t p = 0;
  explicit Reader(const std::string& s) : d(s) {}
  void need(size_t n) {
    if (n > d.size() - p) throw std::runtime_error("kvstore: truncated frame");
  }
  uint8_t u8() { need(1); return (uint8_t)d[p++]; }
  uint32_t u32() { need(4); uint32_t v; memcpy(&v, d.data() + p, 4); p += 4; return v; }
  double f64() { need(8); double v; memcpy(&v, d.data() + p, 8); p += 8; return v; }
  std::string str() { uint32_t n = u32(); need(n); std::string s = d.substr(p, n); p += n; return s; }
};

inline bool send_all(int fd, const char* b, size_t n) {
  while (n) {
    ssize_t k = ::send(fd, b, n, MSG_NOSIGNAL);
    if (k <= 0) return false;
    b += k;
    n -= (size_t)k;
  }
  return true;
}
inline bool recv_all(int fd, char* b, size_t n) {
  while (n) {
    ssize_t k = ::recv(fd, b, n, 0);
    if (k <= 0) return false;
    b += k;
    n -= (size_t)k;
  }
  return true;
}
inline bool send_frame(int fd, const std::string& payload) {
  uint32_t n = (uint32_t)payload.size();
  return send_all(fd, (const char*)&n, 4) && send_all(fd, payload.data(), payload.size());
}
inline bool recv_frame(int fd, std::string& out) {
  uint32_t n;
  if (!recv_all(fd, (char*)&n, 4)) return false;
  if (n > (1u << 30)) return false;
  out.resize(n);
  return n == 0 || recv_all(fd, &out[0], n);
}

struct Record {
  std::string value;
  double expiration;
  std::string owner;
};

using Entry = std::tuple<std::string, std::string, double>;  // (subkey, value, expiration)

class Store {
 public:
  bool store(const std::string& key, const std::string& sub, const std::string& val, double exp,
             const std::string& owner) {
    std::lock_guard<std::mutex> g(mu_);
    const double t = now_s();
    auto& m = data_[key];
    auto it = m.find(sub);
    if (it != m.end() && it->second.expiration > t) {
      if (!it->second.owner.empty() && it->second.owner != owner) return false;  // someone else's subkey
      if (exp < it->second.expiration) return false;  // a fresher value is already stored
    }
    m[sub] = Record{val, exp, owner};
    cv_.notify_all();
    return true;
  }
  std::vector<Entry> get(const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<Entry> out;
    auto it = data_.find(key);
    if (it == data_.end()) return out;
    const double t = now_s();
    for (auto r = it->second.begin(); r != it->second.end();) {
      if (r->second.expiration <= t) {
        r = it->second.erase(r);
      } else {
        out.emplace_back(r->first, r->second.value, r->second.expiration);
        ++r;
      }
    }
    if (it->second.empty()) data_.erase(it);  // do not keep dead keys around forever
    return out;
  }
  void del(const std::string& key) {
    std::lock_guard<std::mutex> g(mu_);
    data_.erase(key);
  }
  std::vector<std::string> keys(const std::string& prefix) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::string> out;
    for (auto& kv : data_)
      if (kv.first.compare(0, prefix.size(), prefix) == 0) out.push_back(kv.first);
    return out;
  }
  uint32_t wait(const std::string& key, uint32_t count, double timeout) {
    std::unique_lock<std::mutex> g(mu_);
    // system_clock deadline: libstdc++ maps it to pthread_cond_timedwait (a steady_clock deadline
    // becomes pthread_cond_clockwait, which ThreadSanitizer does not intercept and then reports as
    // a double lock). The WAIT timeouts are seconds long, so wall-clock adjustments do not matter.
    const auto deadline = std::chrono::system_clock::now() +
                          std::chrono::duration_cast<std::chrono::system_clock::duration>(std::chrono::duration<double>(timeout));
    while (true) {
      uint32_t live = 0;
      auto it = data_.find(key);
      if (it != data_.end()) {
        const double t = now_s();
        for (auto& r : it->second)
          if (r.second.expiration > t) ++live;
      }
      if (live >= count || closing_) return live;
      if (cv_.wait_until(g, deadline) == std::cv_status::timeout) return live;
    }
  }
  // Server shutdown: every pending and future WAIT returns immediately with its current count.
  void close() {
    std::lock_guard<std::mutex> g(mu_);
    closing_ = true;
    cv_.notify_all();
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  bool closing_ = false;
  std::map<std::string, std::map<std::string, Record>> data_;
};

inline std::string handle(Store& st, const std::string& req) {
  Reader r(req);
  Buf out;
  const uint8_t op = r.u8();
  switch (op) {
    case OP_STORE: {
      std::string key = r.str(), sub = r.str(), val = r.str();
      double exp = r.f64();
      std::string owner = r.str();
      out.u8(st.store(key, sub, val, exp, owner) ? 1 : 0);
      break;
    }
    case OP_GET: {
      auto v = st.get(r.str());
      out.u32((uint32_t)v.size());
      for (auto& t : v) {
        out.str(std::get<0>(t));
        out.str(std::get<1>(t));
        out.f64(std::get<2>(t));
      }
      break;
    }
    case OP_DELETE: st.del(r.str()); out.u8(1); break;
    case OP_KEYS: {
      auto v = st.keys(r.str());
      out.u32((uint32_t)v.size());
      for (auto& k : v) out.str(k);
      break;
    }
    case OP_PING: out.u8(1); break;
    case OP_WAIT: {
      std::string key = r.str();
      uint32_t cnt = r.u32();
      double to = r.f64();
      out.u32(st.wait(key, cnt, to));
      break;
    }
    default: throw std::runtime_error("kvstore: bad opcode");
  }
  return out.d;
}

// One thread per connection (a node has at most a few dozen peers). A connection's fd is closed
// only by its own worker, under cmu_, after it left the live set: stop() never shuts down a
// descriptor number the kernel may already have handed to someone else. Finished workers are
// joined by the acceptor, so a long-lived server with reconnecting peers does not accumulate them.
class KVServer {
 public:
  KVServer(const std::string& host, int port) {
    fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd_ < 0) throw std::runtime_error("kvstore: socket() failed");
    int one = 1;
    setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) {
      ::close(fd_);
      throw std::runtime_error("kvstore: bad host " + host);
    }
    if (::bind(fd_, (sockaddr*)&a, sizeof(a)) != 0) {
      ::close(fd_);
      throw std::runtime_error("kvstore: bind failed on " + host + ":" + std::to_string(port));
    }
    ::listen(fd_, 128);
    socklen_t len = sizeof(a);
    getsockname(fd_, (sockaddr*)&a, &len);
    port_ = ntohs(a.sin_port);
    running_ = true;
    acceptor_ = std::thread([this] { loop(); });
  }
  ~KVServer() { stop(); }
  KVServer(const KVServer&) = delete;
  KVServer& operator=(const KVServer&) = delete;
  int port() const { return port_; }
  void stop() {
    if (!running_.exchange(false)) return;
    ::shutdown(fd_, SHUT_RDWR);  // wakes accept()
    if (acceptor_.joinable()) acceptor_.join();
    ::close(fd_);
    std::map<uint64_t, std::thread> ws;
    {
      std::lock_guard<std::mutex> g(cmu_);
      for (int c : live_) ::shutdown(c, SHUT_RDWR);  // wakes recv() in every worker
      ws.swap(workers_);
      finished_.clear();
    }
    st_.close();  // wakes workers parked in WAIT
    for (auto& w : ws)
      if (w.second.joinable()) w.second.join();
  }
  Store& store() { return st_; }
  size_t live_connections() {
    std::lock_guard<std::mutex> g(cmu_);
    return live_.size();
  }

 private:
  void loop() {
    while (running_) {
      int c = ::accept(fd_, nullptr, nullptr);
      if (c < 0) {
        if (!running_) break;
        continue;
      }
      int one = 1;
      setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      std::vector<std::thread> done;
      {
        std::lock_guard<std::mutex> g(cmu_);
        if (!running_) {  // stop() already swept the live set
          ::close(c);
          break;
        }
        for (uint64_t id : finished_) {
          auto it = workers_.find(id);
          if (it != workers_.end()) {
            done.push_back(std::move(it->second));
            workers_.erase(it);
          }
        }
        finished_.clear();
        live_.insert(c);
        const uint64_t id = next_id_++;
        workers_.emplace(id, std::thread([this, c, id] { serve(c, id); }));
      }
      for (auto& t : done) t.join();  // already returned from serve()
    }
  }
  void serve(int c, uint64_t id) {
    std::string req;
    while (running_ && recv_frame(c, req)) {
      std::string rep;
      try {
        rep = handle(st_, req);
      } catch (const std::exception&) {
        break;
      }
      if (!send_frame(c, rep)) break;
    }
    std::lock_guard<std::mutex> g(cmu_);
    live_.erase(c);
    ::close(c);
    finished_.push_back(id);
  }
  int fd_ = -1, port_ = 0;
  std::atomic<bool> running_{false};
  std::thread acceptor_;
  std::mutex cmu_;
  std::set<int> live_;
  std::map<uint64_t, std::thread> workers_;
  std::vector<uint64_t> finished_;
  uint64_t next_id_ = 0;
  Store st_;
};

// Blocking client; one request in flight per client (calls are serialised by mu_).
class ClientCore {
 public:
  ClientCore(const std::string& host, int port, double connect_timeout) : host_(host), port_(port) {
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(connect_timeout);
    while (true) {
      if (try_connect()) break;
      if (std::chrono::steady_clock::now() > deadline)
        throw std::runtime_error("kvstore: cannot connect to " + host + ":" + std::to_string(port));
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
  }
  ~ClientCore() {
    if (fd_ >= 0) ::close(fd_);
  }
  ClientCore(const ClientCore&) = delete;
  ClientCore& operator=(const ClientCore&) = delete;

  bool store(const std::string& key, const std::string& sub, const std::string& val, double exp,
             const std::string& owner) {
    Buf b;
    b.u8(OP_STORE);
    b.str(key);
    b.str(sub);
    b.str(val);
    b.f64(exp);
    b.str(owner);
    std::string rep = call(b.d);
    return Reader(rep).u8() == 1;
  }
  std::vector<Entry> get(const std::string& key) {
    Buf b;
    b.u8(OP_GET);
    b.str(key);
    std::string rep = call(b.d);
    Reader r(rep);
    uint32_t n = r.u32();
    std::vector<Entry> out;
    out.reserve(n);
    for (uint32_t i = 0; i < n; ++i) {
      std::string sub = r.str(), val = r.str();
      double exp = r.f64();
      out.emplace_back(std::move(sub), std::move(val), exp);
    }
    return out;
  }
  void del(const std::string& key) {
    Buf b;
    b.u8(OP_DELETE);
    b.str(key);
    call(b.d);
  }
  std::vector<std::string> keys(const std::string& prefix) {
    Buf b;
    b.u8(OP_KEYS);
    b.str(prefix);
    std::string rep = call(b.d);
    Reader r(rep);
    uint32_t n = r.u32();
    std::vector<std::string> out;
    for (uint32_t i = 0; i < n; ++i) out.push_back(r.str());
    return out;
  }
  bool ping() {
    Buf b;
    b.u8(OP_PING);
    std::string rep = call(b.d);
    return Reader(rep).u8() == 1;
  }
  uint32_t wait(const std::string& key, uint32_t count, double timeout) {
    Buf b;
    b.u8(OP_WAIT);
    b.str(key);
    b.u32(count);
    b.f64(timeout);
    std::string rep = call(b.d);
    return Reader(rep).u32();
  }

 private:
  bool try_connect() {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host_.c_str(), std::to_string(port_).c_str(), &hints, &res) != 0) return false;
    int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
    bool ok = fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0;
    freeaddrinfo(res);
    if (!ok) {
      if (fd >= 0) ::close(fd);
      return false;
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    fd_ = fd;
    return true;
  }
  std::string call(const std::string& req) {
    std::lock_guard<std::mutex> g(mu_);
    std::string rep;
    if (fd_ < 0 || !send_frame(fd_, req) || !recv_frame(fd_, rep)) {
      // one reconnect attempt (server restarted / connection dropped)
      if (fd_ >= 0) ::close(fd_);
      fd_ = -1;
      if (!try_connect() || !send_frame(fd_, req) || !recv_frame(fd_, rep))
        throw std::runtime_error("kvstore: connection lost");
    }
    return rep;
  }
  std::string host_;
  int port_;
  int fd_ = -1;
  std::mutex mu_;
};

}  // namespace dalle_kv
