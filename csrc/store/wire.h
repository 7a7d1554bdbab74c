// Socket + framing helpers shared by the TCP store and the host ring backend.
#pragma once

#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>

#include "../common.h"

namespace ringdp {
namespace wire {

struct Writer {
  std::string buf;
  void u8(uint8_t v) { buf.push_back(static_cast<char>(v)); }
  void u32(uint32_t v) { buf.append(reinterpret_cast<const char*>(&v), 4); }
  void i64(int64_t v) { buf.append(reinterpret_cast<const char*>(&v), 8); }
  void str(const std::string& s) {
    u32(static_cast<uint32_t>(s.size()));
    buf.append(s);
  }
};

struct Reader {
  std::string buf;  // owned: callers often construct a Reader from a temporary reply
  size_t pos = 0;
  explicit Reader(std::string b) : buf(std::move(b)) {}
  void need(size_t n) {
    RINGDP_CHECK(pos + n <= buf.size(), "wire: truncated message");
  }
  uint8_t u8() {
    need(1);
    return static_cast<uint8_t>(buf[pos++]);
  }
  uint32_t u32() {
    need(4);
    uint32_t v;
    std::memcpy(&v, buf.data() + pos, 4);
    pos += 4;
    return v;
  }
  int64_t i64() {
    need(8);
    int64_t v;
    std::memcpy(&v, buf.data() + pos, 8);
    pos += 8;
    return v;
  }
  std::string str() {
    uint32_t n = u32();
    need(n);
    std::string s = buf.substr(pos, n);
    pos += n;
    return s;
  }
};

inline void send_all(int fd, const void* data, size_t n) {
  const char* p = static_cast<const char*>(data);
  while (n > 0) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        pollfd pfd{fd, POLLOUT, 0};
        ::poll(&pfd, 1, 1000);
        continue;
      }
      throw RingdpError(strcat_all("[ringdp] send failed: ", strerror(errno)));
    }
    p += w;
    n -= static_cast<size_t>(w);
  }
}

inline void recv_all(int fd, void* data, size_t n, std::chrono::milliseconds timeout) {
  char* p = static_cast<char*>(data);
  auto deadline = Clock::now() + timeout;
  while (n > 0) {
    auto left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now());
    if (left.count() <= 0) throw TimeoutError("[ringdp] recv timed out (peer unresponsive)");
    pollfd pfd{fd, POLLIN, 0};
    int pr = ::poll(&pfd, 1, static_cast<int>(std::min<int64_t>(left.count(), 1000)));
    if (pr < 0 && errno != EINTR) throw RingdpError(strcat_all("[ringdp] poll: ", strerror(errno)));
    if (pr <= 0) continue;
    ssize_t r = ::recv(fd, p, n, 0);
    if (r == 0) throw RingdpError("[ringdp] connection closed by peer");
    if (r < 0) {
      if (errno == EINTR || errno == EAGAIN || errno == EWOULDBLOCK) continue;
      throw RingdpError(strcat_all("[ringdp] recv failed: ", strerror(errno)));
    }
    p += r;
    n -= static_cast<size_t>(r);
  }
}

inline void send_frame(int fd, const std::string& payload) {
  uint32_t len = static_cast<uint32_t>(payload.size());
  std::string out(reinterpret_cast<const char*>(&len), 4);
  out += payload;
  send_all(fd, out.data(), out.size());
}

inline std::string recv_frame(int fd, std::chrono::milliseconds timeout) {
  uint32_t len = 0;
  recv_all(fd, &len, 4, timeout);
  std::string payload(len, '\0');
  if (len) recv_all(fd, payload.data(), len, timeout);
  return payload;
}

inline int connect_once(const std::string& host, int port) {
  addrinfo hints{};
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  std::string port_s = std::to_string(port);
  if (::getaddrinfo(host.c_str(), port_s.c_str(), &hints, &res) != 0 || !res) return -1;
  int fd = -1;
  for (addrinfo* ai = res; ai; ai = ai->ai_next) {
    fd = ::socket(ai->ai_family, ai->ai_socktype, ai->ai_protocol);
    if (fd < 0) continue;
    if (::connect(fd, ai->ai_addr, ai->ai_addrlen) == 0) break;
    ::close(fd);
    fd = -1;
  }
  ::freeaddrinfo(res);
  if (fd >= 0) {
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  }
  return fd;
}

inline int connect_with_retry(const std::string& host, int port,
                              std::chrono::milliseconds timeout) {
  auto deadline = Clock::now() + timeout;
  int backoff_ms = 5;
  while (true) {
    int fd = connect_once(host, port);
    if (fd >= 0) return fd;
    if (Clock::now() > deadline)
      throw TimeoutError(strcat_all("[ringdp] could not connect to ", host, ":", port,
                                    " within ", timeout.count(), " ms"));
    std::this_thread::sleep_for(std::chrono::milliseconds(backoff_ms));
    backoff_ms = std::min(backoff_ms * 2, 200);
  }
}

}  // namespace wire
}  // namespace ringdp
