// ringdp TCP store: length-prefixed binary protocol, poll()-driven single-thread server.
//
// Behavioural parity with c10d TCPStore (c10d/TCPStore.hpp:73): rank 0
// hosts the daemon, clients retry the connection until the timeout, `get`/`wait` block on the
// server side (waiters are parked until the key appears or their deadline passes), `add`
// keeps decimal text so `get` after `add` returns "N".
#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstring>
#include <map>
#include <set>

#include "store.h"
#include "wire.h"

namespace ringdp {

namespace {

enum Cmd : uint8_t {
  kSet = 1,
  kGet = 2,
  kAdd = 3,
  kCas = 4,
  kCheck = 5,
  kWait = 6,
  kDelete = 7,
  kNumKeys = 8,
  kPing = 9,
};

enum Status : uint8_t { kOk = 0, kTimeout = 1 };

}  // namespace

class TCPStoreServer {
 public:
  explicit TCPStoreServer(int port) {
    listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    RINGDP_CHECK(listen_fd_ >= 0, "socket(): ", strerror(errno));
    int one = 1;
    ::setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in addr{};
    addr.sin_family = AF_INET;
    addr.sin_addr.s_addr = htonl(INADDR_ANY);
    addr.sin_port = htons(static_cast<uint16_t>(port));
    if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0) {
      int e = errno;
      ::close(listen_fd_);
      throw RingdpError(strcat_all("[ringdp] TCPStore bind to port ", port,
                                   " failed: ", strerror(e)));
    }
    RINGDP_CHECK(::listen(listen_fd_, 1024) == 0, "listen(): ", strerror(errno));
    socklen_t len = sizeof(addr);
    ::getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&addr), &len);
    port_ = ntohs(addr.sin_port);
    RINGDP_CHECK(::pipe(wake_) == 0, "pipe(): ", strerror(errno));
    thread_ = std::thread([this] { loop(); });
  }

  ~TCPStoreServer() {
    stop_.store(true);
    char c = 1;
    (void)!::write(wake_[1], &c, 1);
    if (thread_.joinable()) thread_.join();
    for (auto& kv : inbuf_) ::close(kv.first);
    ::close(listen_fd_);
    ::close(wake_[0]);
    ::close(wake_[1]);
  }

  int port() const { return port_; }

 private:
  struct Waiter {
    int fd;
    std::vector<std::string> keys;
    int64_t deadline_us;
    bool is_get;
  };

  void loop() {
    std::vector<pollfd> fds;
    while (!stop_.load()) {
      fds.clear();
      fds.push_back({listen_fd_, POLLIN, 0});
      fds.push_back({wake_[0], POLLIN, 0});
      for (auto& kv : inbuf_) fds.push_back({kv.first, POLLIN, 0});
      int timeout_ms = 1000;
      int64_t now = now_us();
      for (auto& w : waiters_) {
        int64_t ms = std::max<int64_t>(0, (w.deadline_us - now) / 1000 + 1);
        timeout_ms = static_cast<int>(std::min<int64_t>(timeout_ms, ms));
      }
      int n = ::poll(fds.data(), fds.size(), timeout_ms);
      if (n < 0 && errno != EINTR) break;
      if (stop_.load()) break;
      if (n > 0) {
        if (fds[0].revents & POLLIN) accept_client();
        for (size_t i = 2; i < fds.size(); ++i) {
          if (fds[i].revents & (POLLIN | POLLHUP | POLLERR)) {
            if (!read_client(fds[i].fd)) drop_client(fds[i].fd);
          }
        }
      }
      expire_waiters();
    }
  }

  void accept_client() {
    int fd = ::accept(listen_fd_, nullptr, nullptr);
    if (fd < 0) return;
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    inbuf_[fd] = std::string();
  }

  void drop_client(int fd) {
    ::close(fd);
    inbuf_.erase(fd);
    waiters_.erase(std::remove_if(waiters_.begin(), waiters_.end(),
                                  [fd](const Waiter& w) { return w.fd == fd; }),
                   waiters_.end());
  }

  bool read_client(int fd) {
    char buf[65536];
    ssize_t r = ::recv(fd, buf, sizeof(buf), 0);
    if (r <= 0) return false;
    std::string& in = inbuf_[fd];
    in.append(buf, static_cast<size_t>(r));
    while (in.size() >= 4) {
      uint32_t len;
      std::memcpy(&len, in.data(), 4);
      if (in.size() < 4 + static_cast<size_t>(len)) break;
      std::string frame = in.substr(4, len);
      in.erase(0, 4 + len);
      if (!handle(fd, frame)) return false;
    }
    return true;
  }

  void reply(int fd, const std::string& payload) { wire::send_frame(fd, payload); }

  bool all_present(const std::vector<std::string>& keys) const {
    for (auto& k : keys)
      if (data_.find(k) == data_.end()) return false;
    return true;
  }

  void notify(const std::string& key) {
    for (auto it = waiters_.begin(); it != waiters_.end();) {
      bool relevant = std::find(it->keys.begin(), it->keys.end(), key) != it->keys.end();
      if (relevant && all_present(it->keys)) {
        wire::Writer w;
        w.u8(kOk);
        if (it->is_get) w.str(data_[it->keys[0]]);
        reply(it->fd, w.buf);
        it = waiters_.erase(it);
      } else {
        ++it;
      }
    }
  }

  void expire_waiters() {
    int64_t now = now_us();
    for (auto it = waiters_.begin(); it != waiters_.end();) {
      if (it->deadline_us <= now) {
        wire::Writer w;
        w.u8(kTimeout);
        reply(it->fd, w.buf);
        it = waiters_.erase(it);
      } else {
        ++it;
      }
    }
  }

  bool handle(int fd, const std::string& frame) {
    wire::Reader r(frame);
    uint8_t cmd = r.u8();
    wire::Writer w;
    switch (cmd) {
      case kSet: {
        std::string key = r.str();
        data_[key] = r.str();
        w.u8(kOk);
        reply(fd, w.buf);
        notify(key);
        return true;
      }
      case kGet: {
        std::string key = r.str();
        int64_t timeout_ms = r.i64();
        auto it = data_.find(key);
        if (it != data_.end()) {
          w.u8(kOk);
          w.str(it->second);
          reply(fd, w.buf);
        } else {
          waiters_.push_back({fd, {key}, now_us() + timeout_ms * 1000, true});
        }
        return true;
      }
      case kAdd: {
        std::string key = r.str();
        int64_t delta = r.i64();
        int64_t cur = 0;
        auto it = data_.find(key);
        if (it != data_.end() && !it->second.empty()) cur = std::stoll(it->second);
        cur += delta;
        data_[key] = std::to_string(cur);
        w.u8(kOk);
        w.i64(cur);
        reply(fd, w.buf);
        notify(key);
        return true;
      }
      case kCas: {
        std::string key = r.str();
        std::string expected = r.str();
        std::string desired = r.str();
        auto it = data_.find(key);
        std::string out;
        bool changed = false;
        if (it == data_.end()) {
          if (expected.empty()) {
            data_[key] = desired;
            out = desired;
            changed = true;
          } else {
            out = expected;
          }
        } else if (it->second == expected) {
          it->second = desired;
          out = desired;
          changed = true;
        } else {
          out = it->second;
        }
        w.u8(kOk);
        w.str(out);
        reply(fd, w.buf);
        if (changed) notify(key);
        return true;
      }
      case kCheck: {
        uint32_t n = r.u32();
        std::vector<std::string> keys;
        for (uint32_t i = 0; i < n; ++i) keys.push_back(r.str());
        w.u8(kOk);
        w.u8(all_present(keys) ? 1 : 0);
        reply(fd, w.buf);
        return true;
      }
      case kWait: {
        uint32_t n = r.u32();
        std::vector<std::string> keys;
        for (uint32_t i = 0; i < n; ++i) keys.push_back(r.str());
        int64_t timeout_ms = r.i64();
        if (all_present(keys)) {
          w.u8(kOk);
          reply(fd, w.buf);
        } else {
          waiters_.push_back({fd, keys, now_us() + timeout_ms * 1000, false});
        }
        return true;
      }
      case kDelete: {
        std::string key = r.str();
        bool erased = data_.erase(key) > 0;
        w.u8(kOk);
        w.u8(erased ? 1 : 0);
        reply(fd, w.buf);
        return true;
      }
      case kNumKeys: {
        w.u8(kOk);
        w.i64(static_cast<int64_t>(data_.size()));
        reply(fd, w.buf);
        return true;
      }
      case kPing: {
        w.u8(kOk);
        reply(fd, w.buf);
        return true;
      }
      default:
        return false;
    }
  }

  int listen_fd_ = -1;
  int port_ = 0;
  int wake_[2] = {-1, -1};
  std::atomic<bool> stop_{false};
  std::thread thread_;
  std::map<int, std::string> inbuf_;
  std::map<std::string, std::string> data_;
  std::vector<Waiter> waiters_;
};

TCPStore::TCPStore(const std::string& host, int port, bool is_master,
                   std::chrono::milliseconds timeout, int world_size, bool wait_for_workers)
    : Store(timeout), host_(host), port_(port) {
  if (is_master) {
    server_ = std::make_unique<TCPStoreServer>(port);
    port_ = server_->port();
  }
  fd_ = wire::connect_with_retry(is_master ? "127.0.0.1" : host_, port_, timeout_);
  if (wait_for_workers && world_size > 0) {
    // Every rank checks in; the master waits until all have (c10d TCPStore semantics).
    add("__ringdp_store_init", 1);
    if (is_master) {
      auto deadline = Clock::now() + timeout_;
      while (true) {
        int64_t n = add("__ringdp_store_init", 0);
        if (n >= world_size) break;
        if (Clock::now() > deadline)
          throw TimeoutError(strcat_all("[ringdp] TCPStore: timed out waiting for ", world_size,
                                        " workers (", n, " joined)"));
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
      }
    }
  }
}

TCPStore::~TCPStore() {
  if (fd_ >= 0) ::close(fd_);
  server_.reset();
}

std::string TCPStore::request(const std::string& payload, std::chrono::milliseconds timeout) {
  std::lock_guard<std::mutex> lk(mu_);
  wire::send_frame(fd_, payload);
  // The server enforces the logical timeout; allow slack for the reply to arrive.
  return wire::recv_frame(fd_, timeout + std::chrono::milliseconds(30000));
}

void TCPStore::set(const std::string& key, const std::string& value) {
  wire::Writer w;
  w.u8(kSet);
  w.str(key);
  w.str(value);
  request(w.buf, timeout_);
}

std::string TCPStore::get(const std::string& key) {
  wire::Writer w;
  w.u8(kGet);
  w.str(key);
  w.i64(timeout_.count());
  wire::Reader r(request(w.buf, timeout_));
  if (r.u8() != kOk)
    throw TimeoutError(strcat_all("[ringdp] TCPStore get('", key, "') timed out after ",
                                  timeout_.count(), " ms"));
  return r.str();
}

int64_t TCPStore::add(const std::string& key, int64_t delta) {
  wire::Writer w;
  w.u8(kAdd);
  w.str(key);
  w.i64(delta);
  wire::Reader r(request(w.buf, timeout_));
  r.u8();
  return r.i64();
}

std::string TCPStore::compare_set(const std::string& key, const std::string& expected,
                                  const std::string& desired) {
  wire::Writer w;
  w.u8(kCas);
  w.str(key);
  w.str(expected);
  w.str(desired);
  wire::Reader r(request(w.buf, timeout_));
  r.u8();
  return r.str();
}

bool TCPStore::check(const std::vector<std::string>& keys) {
  wire::Writer w;
  w.u8(kCheck);
  w.u32(static_cast<uint32_t>(keys.size()));
  for (auto& k : keys) w.str(k);
  wire::Reader r(request(w.buf, timeout_));
  r.u8();
  return r.u8() != 0;
}

void TCPStore::wait(const std::vector<std::string>& keys, std::chrono::milliseconds timeout) {
  wire::Writer w;
  w.u8(kWait);
  w.u32(static_cast<uint32_t>(keys.size()));
  for (auto& k : keys) w.str(k);
  w.i64(timeout.count());
  wire::Reader r(request(w.buf, timeout));
  if (r.u8() != kOk) {
    std::string names;
    for (auto& k : keys) names += k + " ";
    throw TimeoutError(strcat_all("[ringdp] TCPStore wait timed out after ", timeout.count(),
                                  " ms for keys: ", names));
  }
}

bool TCPStore::delete_key(const std::string& key) {
  wire::Writer w;
  w.u8(kDelete);
  w.str(key);
  wire::Reader r(request(w.buf, timeout_));
  r.u8();
  return r.u8() != 0;
}

int64_t TCPStore::num_keys() {
  wire::Writer w;
  w.u8(kNumKeys);
  wire::Reader r(request(w.buf, timeout_));
  r.u8();
  return r.i64();
}

}  // namespace ringdp
