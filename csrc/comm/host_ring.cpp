// Host ring backend: CPU tensor collectives over a TCP full mesh.
//
// Ring all-reduce = reduce-scatter + all-gather over the logical ring rank -> rank+1, i.e. the
// algorithm the reference's README explains (ref/README.md:3-20): every
// rank sends 2(N-1)/N of the buffer regardless of N.  Each message carries a header
// {seq, op, bytes}; a mismatch is reported as a collective desync (the c10d ProcessGroupWrapper /
// TORCH_DISTRIBUTED_DEBUG=DETAIL fingerprint) instead of silently corrupting data.
#include "host_ring.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <c10/util/BFloat16.h>
#include <c10/util/Half.h>

#include <cstring>

#include "../store/wire.h"

namespace ringdp {

const char* op_name(OpType t) {
  switch (t) {
    case OpType::ALLREDUCE: return "allreduce";
    case OpType::BROADCAST: return "broadcast";
    case OpType::ALLGATHER: return "allgather";
    case OpType::ALLGATHER_BASE: return "allgather_into_tensor";
    case OpType::REDUCE_SCATTER_BASE: return "reduce_scatter_tensor";
    case OpType::REDUCE: return "reduce";
    case OpType::GATHER: return "gather";
    case OpType::SCATTER: return "scatter";
    case OpType::ALLTOALL_BASE: return "all_to_all_single";
    case OpType::SEND: return "send";
    case OpType::RECV: return "recv";
    case OpType::BARRIER: return "barrier";
    case OpType::COALESCED: return "coalesced";
    case OpType::GRAPH_REPLAY: return "graph_replay";
  }
  return "unknown";
}

// ------------------------------------------------------------------ HostWork
void HostWork::wait(bool /*blocking*/) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [&] { return done_.load(); });
  if (err_) std::rethrow_exception(err_);
}

void HostWork::finish(std::exception_ptr err) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    err_ = err;
    duration_us_ = static_cast<double>(now_us() - start_us_);
    done_.store(true);
  }
  cv_.notify_all();
}

// ------------------------------------------------------------------ reductions
namespace {

template <typename T>
void reduce_typed(T* d, const T* s, int64_t n, ReduceOp op) {
  switch (op) {
    case ReduceOp::SUM:
    case ReduceOp::AVG:
      for (int64_t i = 0; i < n; ++i) d[i] = static_cast<T>(d[i] + s[i]);
      break;
    case ReduceOp::PRODUCT:
      for (int64_t i = 0; i < n; ++i) d[i] = static_cast<T>(d[i] * s[i]);
      break;
    case ReduceOp::MIN:
      for (int64_t i = 0; i < n; ++i) d[i] = s[i] < d[i] ? s[i] : d[i];
      break;
    case ReduceOp::MAX:
      for (int64_t i = 0; i < n; ++i) d[i] = s[i] > d[i] ? s[i] : d[i];
      break;
    default:
      throw RingdpError("[ringdp] bitwise reduce ops require an integer dtype");
  }
}

template <typename T>
void reduce_int(T* d, const T* s, int64_t n, ReduceOp op) {
  switch (op) {
    case ReduceOp::BAND:
      for (int64_t i = 0; i < n; ++i) d[i] = d[i] & s[i];
      break;
    case ReduceOp::BOR:
      for (int64_t i = 0; i < n; ++i) d[i] = d[i] | s[i];
      break;
    case ReduceOp::BXOR:
      for (int64_t i = 0; i < n; ++i) d[i] = d[i] ^ s[i];
      break;
    default:
      reduce_typed<T>(d, s, n, op);
  }
}

void reduce_bool(bool* d, const bool* s, int64_t n, ReduceOp op) {
  for (int64_t i = 0; i < n; ++i) {
    switch (op) {
      case ReduceOp::SUM:
      case ReduceOp::MAX:
      case ReduceOp::BOR:
      case ReduceOp::AVG:
        d[i] = d[i] || s[i];
        break;
      case ReduceOp::PRODUCT:
      case ReduceOp::MIN:
      case ReduceOp::BAND:
        d[i] = d[i] && s[i];
        break;
      case ReduceOp::BXOR:
        d[i] = d[i] != s[i];
        break;
    }
  }
}

}  // namespace

void host_reduce_raw(void* dst, const void* src, int64_t n, at::ScalarType dtype, ReduceOp op) {
  switch (dtype) {
    case at::kFloat: reduce_typed(static_cast<float*>(dst), static_cast<const float*>(src), n, op); break;
    case at::kDouble: reduce_typed(static_cast<double*>(dst), static_cast<const double*>(src), n, op); break;
    case at::kHalf: reduce_typed(static_cast<c10::Half*>(dst), static_cast<const c10::Half*>(src), n, op); break;
    case at::kBFloat16: reduce_typed(static_cast<c10::BFloat16*>(dst), static_cast<const c10::BFloat16*>(src), n, op); break;
    case at::kInt: reduce_int(static_cast<int32_t*>(dst), static_cast<const int32_t*>(src), n, op); break;
    case at::kLong: reduce_int(static_cast<int64_t*>(dst), static_cast<const int64_t*>(src), n, op); break;
    case at::kShort: reduce_int(static_cast<int16_t*>(dst), static_cast<const int16_t*>(src), n, op); break;
    case at::kChar: reduce_int(static_cast<int8_t*>(dst), static_cast<const int8_t*>(src), n, op); break;
    case at::kByte: reduce_int(static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), n, op); break;
    case at::kBool: reduce_bool(static_cast<bool*>(dst), static_cast<const bool*>(src), n, op); break;
    default:
      throw RingdpError(strcat_all("[ringdp] host reduce: unsupported dtype ", c10::toString(dtype)));
  }
}

void host_reduce_inplace(at::Tensor& dst, const at::Tensor& src, ReduceOp op) {
  host_reduce_raw(dst.data_ptr(), src.data_ptr(), dst.numel(), dst.scalar_type(), op);
}

namespace {

void finish_avg(at::Tensor& t, int size) {
  if (at::isFloatingType(t.scalar_type())) {
    t.div_(static_cast<double>(size));
  } else if (t.scalar_type() != at::kBool) {
    t.div_(size, "trunc");
  }
}

struct MsgHeader {
  uint64_t seq;
  uint32_t op;
  uint32_t magic;
  uint64_t bytes;
};
constexpr uint32_t kMagic = 0x52494e47;  // "RING"

void set_nonblocking(int fd) {
  int fl = ::fcntl(fd, F_GETFL, 0);
  ::fcntl(fd, F_SETFL, fl | O_NONBLOCK);
}

std::string local_ip_for(const std::string& hint) {
  if (hint.empty() || hint == "127.0.0.1" || hint == "localhost") return "127.0.0.1";
  int fd = ::socket(AF_INET, SOCK_DGRAM, 0);
  if (fd < 0) return "127.0.0.1";
  addrinfo hints{};
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_DGRAM;
  addrinfo* res = nullptr;
  std::string ip = "127.0.0.1";
  if (::getaddrinfo(hint.c_str(), "9", &hints, &res) == 0 && res) {
    if (::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
      sockaddr_in local{};
      socklen_t len = sizeof(local);
      if (::getsockname(fd, reinterpret_cast<sockaddr*>(&local), &len) == 0) {
        char buf[INET_ADDRSTRLEN];
        ::inet_ntop(AF_INET, &local.sin_addr, buf, sizeof(buf));
        ip = buf;
      }
    }
    ::freeaddrinfo(res);
  }
  ::close(fd);
  return ip;
}

at::Tensor contig(const at::Tensor& t) {
  RINGDP_CHECK(t.device().is_cpu(), "host_ring backend expects CPU tensors, got ", t.device());
  return t.is_contiguous() ? t : t.contiguous();
}

}  // namespace

// ------------------------------------------------------------------ construction
HostRingPG::HostRingPG(std::shared_ptr<Store> store, int rank, int size,
                       std::chrono::milliseconds timeout, const std::string& bind_hint)
    : ProcessGroup(rank, size), store_(std::move(store)), timeout_(timeout), bind_hint_(bind_hint) {
  coll_fds_.assign(size, -1);
  p2p_fds_.assign(size, -1);
  if (size > 1) {
    int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
    RINGDP_CHECK(lfd >= 0, "socket(): ", strerror(errno));
    int one = 1;
    ::setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in addr{};
    addr.sin_family = AF_INET;
    addr.sin_addr.s_addr = htonl(INADDR_ANY);
    addr.sin_port = 0;
    RINGDP_CHECK(::bind(lfd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) == 0,
                 "bind(): ", strerror(errno));
    RINGDP_CHECK(::listen(lfd, 4 * size) == 0, "listen(): ", strerror(errno));
    socklen_t len = sizeof(addr);
    ::getsockname(lfd, reinterpret_cast<sockaddr*>(&addr), &len);
    int port = ntohs(addr.sin_port);
    std::string ip = local_ip_for(bind_hint_);
    store_->set("hostring/addr/" + std::to_string(rank), ip + ":" + std::to_string(port));

    // Connect to every lower rank (twice: collective mesh + p2p mesh), accept from higher ranks.
    for (int j = 0; j < rank; ++j) {
      std::string a = store_->get("hostring/addr/" + std::to_string(j));
      auto colon = a.rfind(':');
      std::string host = a.substr(0, colon);
      int p = std::stoi(a.substr(colon + 1));
      for (int mesh = 0; mesh < 2; ++mesh) {
        int fd = wire::connect_with_retry(host, p, timeout_);
        int32_t hello[2] = {rank, mesh};
        wire::send_all(fd, hello, sizeof(hello));
        (mesh == 0 ? coll_fds_ : p2p_fds_)[j] = fd;
      }
    }
    int expected = 2 * (size - 1 - rank);
    for (int k = 0; k < expected; ++k) {
      pollfd pfd{lfd, POLLIN, 0};
      int pr = ::poll(&pfd, 1, static_cast<int>(timeout_.count()));
      RINGDP_CHECK(pr > 0, "host_ring: timed out waiting for peer connections (rank ", rank, ")");
      int fd = ::accept(lfd, nullptr, nullptr);
      RINGDP_CHECK(fd >= 0, "accept(): ", strerror(errno));
      ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      int32_t hello[2];
      wire::recv_all(fd, hello, sizeof(hello), timeout_);
      RINGDP_CHECK(hello[0] > rank && hello[0] < size, "host_ring: bad hello from peer");
      (hello[1] == 0 ? coll_fds_ : p2p_fds_)[hello[0]] = fd;
    }
    ::close(lfd);
    for (int j = 0; j < size; ++j) {
      if (j == rank) continue;
      int bufsz = 4 << 20;
      for (int fd : {coll_fds_[j], p2p_fds_[j]}) {
        ::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &bufsz, sizeof(bufsz));
        ::setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &bufsz, sizeof(bufsz));
        set_nonblocking(fd);
      }
    }
  }
  start_queue(coll_q_);
  start_queue(send_q_);
  start_queue(recv_q_);
}

HostRingPG::~HostRingPG() { shutdown(); }

void HostRingPG::shutdown() {
  if (shut_) return;
  shut_ = true;
  stop_queue(coll_q_);
  stop_queue(send_q_);
  stop_queue(recv_q_);
  for (int fd : coll_fds_)
    if (fd >= 0) ::close(fd);
  for (int fd : p2p_fds_)
    if (fd >= 0) ::close(fd);
  coll_fds_.assign(coll_fds_.size(), -1);
  p2p_fds_.assign(p2p_fds_.size(), -1);
}

void HostRingPG::start_queue(Queue& q) {
  q.th = std::thread([&q] {
    while (true) {
      std::function<void()> task;
      {
        std::unique_lock<std::mutex> lk(q.mu);
        q.cv.wait(lk, [&] { return q.stop || !q.tasks.empty(); });
        if (q.tasks.empty()) return;
        task = std::move(q.tasks.front());
        q.tasks.pop_front();
      }
      task();
      std::lock_guard<std::mutex> lk(q.mu);
      q.done.push_back(std::move(task));  // freed by the caller's thread (see Queue::done)
    }
  });
}

void HostRingPG::stop_queue(Queue& q) {
  {
    std::lock_guard<std::mutex> lk(q.mu);
    q.stop = true;
  }
  q.cv.notify_all();
  if (q.th.joinable()) q.th.join();
  q.done.clear();
}

std::shared_ptr<Work> HostRingPG::enqueue(Queue& q, OpType op, std::function<void(HostWork&)> fn) {
  RINGDP_CHECK(!shut_, "process group has been shut down");
  auto work = std::make_shared<HostWork>(op, next_seq());
  std::vector<std::function<void()>> finished;
  {
    std::lock_guard<std::mutex> lk(q.mu);
    finished.swap(q.done);  // destroyed on this (the caller's) thread, outside the lock
    q.tasks.emplace_back([work, fn = std::move(fn)] {
      try {
        fn(*work);
        work->finish();
      } catch (...) {
        work->finish(std::current_exception());
      }
    });
  }
  q.cv.notify_one();
  return work;
}

// ------------------------------------------------------------------ transport
void HostRingPG::sendrecv(int send_peer, const void* sbuf, size_t sbytes, int recv_peer,
                          void* rbuf, size_t rbytes, uint64_t seq, OpType op) {
  MsgHeader shdr{seq, static_cast<uint32_t>(op), kMagic, sbytes};
  MsgHeader rhdr{};
  const bool do_send = send_peer >= 0;
  const bool do_recv = recv_peer >= 0;
  int sfd = do_send ? coll_fds_[send_peer] : -1;
  int rfd = do_recv ? coll_fds_[recv_peer] : -1;
  size_t s_hdr = 0, s_pay = 0, r_hdr = 0, r_pay = 0;
  auto deadline = Clock::now() + timeout_;
  auto send_done = [&] { return !do_send || (s_hdr == sizeof(shdr) && s_pay == sbytes); };
  auto recv_done = [&] { return !do_recv || (r_hdr == sizeof(rhdr) && r_pay == rbytes); };
  while (!send_done() || !recv_done()) {
    pollfd pfds[2];
    int n = 0;
    int si = -1, ri = -1;
    if (!send_done()) {
      pfds[n] = {sfd, POLLOUT, 0};
      si = n++;
    }
    if (!recv_done()) {
      if (si >= 0 && rfd == sfd) {
        pfds[si].events |= POLLIN;
        ri = si;
      } else {
        pfds[n] = {rfd, POLLIN, 0};
        ri = n++;
      }
    }
    int pr = ::poll(pfds, n, 200);
    if (pr < 0 && errno != EINTR) throw RingdpError(strcat_all("[ringdp] poll: ", strerror(errno)));
    if (Clock::now() > deadline)
      throw TimeoutError(strcat_all("[ringdp] host_ring ", op_name(op), " seq ", seq, " rank ",
                                    rank_, ": timed out after ", timeout_.count(),
                                    " ms exchanging with peers ", send_peer, "/", recv_peer,
                                    " (peer dead or collectives out of sync)"));
    if (pr <= 0) continue;
    if (si >= 0 && (pfds[si].revents & (POLLOUT | POLLERR | POLLHUP))) {
      while (!send_done()) {
        const char* p;
        size_t left;
        if (s_hdr < sizeof(shdr)) {
          p = reinterpret_cast<const char*>(&shdr) + s_hdr;
          left = sizeof(shdr) - s_hdr;
        } else {
          p = static_cast<const char*>(sbuf) + s_pay;
          left = sbytes - s_pay;
        }
        ssize_t w = ::send(sfd, p, left, MSG_NOSIGNAL);
        if (w < 0) {
          if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) break;
          throw RingdpError(strcat_all("[ringdp] host_ring send to rank ", send_peer,
                                       " failed: ", strerror(errno)));
        }
        if (s_hdr < sizeof(shdr))
          s_hdr += static_cast<size_t>(w);
        else
          s_pay += static_cast<size_t>(w);
      }
    }
    if (ri >= 0 && (pfds[ri].revents & (POLLIN | POLLERR | POLLHUP))) {
      while (!recv_done()) {
        char* p;
        size_t left;
        if (r_hdr < sizeof(rhdr)) {
          p = reinterpret_cast<char*>(&rhdr) + r_hdr;
          left = sizeof(rhdr) - r_hdr;
        } else {
          p = static_cast<char*>(rbuf) + r_pay;
          left = rbytes - r_pay;
        }
        ssize_t r = ::recv(rfd, p, left, 0);
        if (r == 0)
          throw RingdpError(strcat_all("[ringdp] host_ring: rank ", recv_peer,
                                       " closed the connection during ", op_name(op), " seq ", seq));
        if (r < 0) {
          if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) break;
          throw RingdpError(strcat_all("[ringdp] host_ring recv from rank ", recv_peer,
                                       " failed: ", strerror(errno)));
        }
        if (r_hdr < sizeof(rhdr)) {
          r_hdr += static_cast<size_t>(r);
          if (r_hdr == sizeof(rhdr)) {
            if (rhdr.magic != kMagic || rhdr.seq != seq || rhdr.op != static_cast<uint32_t>(op) ||
                rhdr.bytes != rbytes) {
              throw RingdpError(strcat_all(
                  "[ringdp] collective desync detected on rank ", rank_, ": expected ",
                  op_name(op), " seq ", seq, " (", rbytes, " B) from rank ", recv_peer, ", got ",
                  rhdr.magic == kMagic ? op_name(static_cast<OpType>(rhdr.op)) : "garbage",
                  " seq ", rhdr.seq, " (", rhdr.bytes, " B)"));
            }
          }
        } else {
          r_pay += static_cast<size_t>(r);
        }
      }
    }
  }
}

void HostRingPG::send_to(int peer, const void* buf, size_t bytes, uint64_t seq, OpType op,
                         const std::vector<int>& mesh) {
  MsgHeader h{seq, static_cast<uint32_t>(op), kMagic, bytes};
  int fd = mesh[peer];
  wire::send_all(fd, &h, sizeof(h));
  if (bytes) wire::send_all(fd, buf, bytes);
}

void HostRingPG::recv_from(int peer, void* buf, size_t bytes, uint64_t seq, OpType op,
                           const std::vector<int>& mesh) {
  MsgHeader h{};
  int fd = mesh[peer];
  wire::recv_all(fd, &h, sizeof(h), timeout_);
  if (h.magic != kMagic || h.op != static_cast<uint32_t>(op) || h.bytes != bytes ||
      (op != OpType::SEND && op != OpType::RECV && h.seq != seq)) {
    throw RingdpError(strcat_all("[ringdp] desync on rank ", rank_, ": expected ", op_name(op),
                                 " (", bytes, " B) from rank ", peer, ", got ",
                                 op_name(static_cast<OpType>(h.op)), " (", h.bytes, " B)"));
  }
  if (bytes) wire::recv_all(fd, buf, bytes, timeout_);
}

// ------------------------------------------------------------------ ring algorithms
void HostRingPG::ring_reduce_scatter(char* data, const std::vector<int64_t>& counts,
                                     const std::vector<int64_t>& offs, at::ScalarType dtype,
                                     size_t esize, ReduceOp op, uint64_t seq, OpType optype) {
  const int n = size_;
  const int next = (rank_ + 1) % n, prev = (rank_ + n - 1) % n;
  int64_t maxc = 0;
  for (auto c : counts) maxc = std::max(maxc, c);
  std::vector<char> tmp(static_cast<size_t>(maxc) * esize);
  for (int s = 0; s < n - 1; ++s) {
    int si = ((rank_ - s - 1) % n + n) % n;
    int ri = ((rank_ - s - 2) % n + n) % n;
    sendrecv(next, data + offs[si] * esize, counts[si] * esize, prev, tmp.data(),
             counts[ri] * esize, seq, optype);
    host_reduce_raw(data + offs[ri] * esize, tmp.data(), counts[ri], dtype, op);
  }
}

void HostRingPG::ring_allgather(char* data, const std::vector<int64_t>& bytes_per_rank,
                                const std::vector<int64_t>& byte_offs, uint64_t seq,
                                OpType optype) {
  const int n = size_;
  const int next = (rank_ + 1) % n, prev = (rank_ + n - 1) % n;
  for (int s = 0; s < n - 1; ++s) {
    int si = ((rank_ - s) % n + n) % n;
    int ri = ((rank_ - s - 1) % n + n) % n;
    sendrecv(next, data + byte_offs[si], bytes_per_rank[si], prev, data + byte_offs[ri],
             bytes_per_rank[ri], seq, optype);
  }
}

void HostRingPG::ring_allreduce(at::Tensor& flat, ReduceOp op, uint64_t seq) {
  const int n = size_;
  if (n == 1) return;
  const int64_t numel = flat.numel();
  const size_t es = flat.element_size();
  std::vector<int64_t> counts(n), offs(n), bcounts(n), boffs(n);
  int64_t base = numel / n, rem = numel % n, o = 0;
  for (int i = 0; i < n; ++i) {
    counts[i] = base + (i < rem ? 1 : 0);
    offs[i] = o;
    o += counts[i];
    bcounts[i] = counts[i] * es;
    boffs[i] = offs[i] * es;
  }
  char* data = static_cast<char*>(flat.data_ptr());
  ring_reduce_scatter(data, counts, offs, flat.scalar_type(), es, op, seq, OpType::ALLREDUCE);
  ring_allgather(data, bcounts, boffs, seq, OpType::ALLREDUCE);
}

void HostRingPG::ring_broadcast(char* data, size_t bytes, int root, uint64_t seq) {
  const int n = size_;
  if (n == 1) return;
  const int next = (rank_ + 1) % n, prev = (rank_ + n - 1) % n;
  // Pipelined chain root -> root+1 -> ... in 1 MiB chunks.
  constexpr size_t kChunk = 1 << 20;
  const bool is_last = next == root;
  for (size_t off = 0; off < bytes || (bytes == 0 && off == 0); off += kChunk) {
    size_t len = std::min(kChunk, bytes - off);
    if (rank_ == root) {
      sendrecv(next, data + off, len, -1, nullptr, 0, seq, OpType::BROADCAST);
    } else {
      sendrecv(-1, nullptr, 0, prev, data + off, len, seq, OpType::BROADCAST);
      if (!is_last) sendrecv(next, data + off, len, -1, nullptr, 0, seq, OpType::BROADCAST);
    }
    if (bytes == 0) break;
  }
}

// ------------------------------------------------------------------ collectives
std::shared_ptr<Work> HostRingPG::allreduce(std::vector<at::Tensor>& tensors, ReduceOp op) {
  auto ts = tensors;
  return enqueue(coll_q_, OpType::ALLREDUCE, [this, ts, op](HostWork& w) mutable {
    for (auto& t : ts) {
      at::Tensor c = contig(t);
      ring_allreduce(c, op, w.seq());
      if (op == ReduceOp::AVG) finish_avg(c, size_);
      if (!c.is_same(t)) t.copy_(c);
    }
    w.outputs_ = ts;
  });
}

std::shared_ptr<Work> HostRingPG::allreduce_coalesced(std::vector<at::Tensor>& tensors,
                                                      ReduceOp op) {
  auto ts = tensors;
  return enqueue(coll_q_, OpType::ALLREDUCE, [this, ts, op](HostWork& w) mutable {
    if (ts.empty()) return;
    std::vector<at::Tensor> flats;
    for (auto& t : ts) flats.push_back(contig(t).view({-1}));
    at::Tensor flat = at::cat(flats);
    ring_allreduce(flat, op, w.seq());
    if (op == ReduceOp::AVG) finish_avg(flat, size_);
    int64_t off = 0;
    for (auto& t : ts) {
      t.copy_(flat.narrow(0, off, t.numel()).view(t.sizes()));
      off += t.numel();
    }
    w.outputs_ = ts;
  });
}

std::shared_ptr<Work> HostRingPG::broadcast(std::vector<at::Tensor>& tensors, int root) {
  RINGDP_CHECK(root >= 0 && root < size_, "broadcast: invalid root ", root);
  auto ts = tensors;
  return enqueue(coll_q_, OpType::BROADCAST, [this, ts, root](HostWork& w) mutable {
    for (auto& t : ts) {
      at::Tensor c = contig(t);
      ring_broadcast(static_cast<char*>(c.data_ptr()), c.nbytes(), root, w.seq());
      if (!c.is_same(t)) t.copy_(c);
    }
    w.outputs_ = ts;
  });
}

std::shared_ptr<Work> HostRingPG::allgather(std::vector<at::Tensor>& outputs,
                                            const at::Tensor& input) {
  RINGDP_CHECK(static_cast<int>(outputs.size()) == size_, "allgather: expected ", size_,
               " output tensors, got ", outputs.size());
  auto outs = outputs;
  at::Tensor in = input;
  return enqueue(coll_q_, OpType::ALLGATHER, [this, outs, in](HostWork& w) mutable {
    at::Tensor c = contig(in);
    const int64_t nb = c.nbytes();
    at::Tensor flat = at::empty({nb * size_}, c.options().dtype(at::kByte));
    char* data = static_cast<char*>(flat.data_ptr());
    std::memcpy(data + nb * rank_, c.data_ptr(), nb);
    std::vector<int64_t> b(size_, nb), o(size_);
    for (int i = 0; i < size_; ++i) o[i] = nb * i;
    if (size_ > 1) ring_allgather(data, b, o, w.seq(), OpType::ALLGATHER);
    for (int i = 0; i < size_; ++i) {
      at::Tensor src = flat.narrow(0, nb * i, nb).view(c.scalar_type()).view(c.sizes());
      outs[i].copy_(src);
    }
    w.outputs_ = outs;
  });
}

std::shared_ptr<Work> HostRingPG::allgather_into_tensor(at::Tensor& output,
                                                        const at::Tensor& input) {
  RINGDP_CHECK(output.numel() == input.numel() * size_,
               "allgather_into_tensor: output numel must be world_size * input numel");
  at::Tensor out = output, in = input;
  return enqueue(coll_q_, OpType::ALLGATHER_BASE, [this, out, in](HostWork& w) mutable {
    at::Tensor c = contig(in);
    at::Tensor o = contig(out);
    const int64_t nb = c.nbytes();
    char* data = static_cast<char*>(o.data_ptr());
    std::memcpy(data + nb * rank_, c.data_ptr(), nb);
    std::vector<int64_t> b(size_, nb), offs(size_);
    for (int i = 0; i < size_; ++i) offs[i] = nb * i;
    if (size_ > 1) ring_allgather(data, b, offs, w.seq(), OpType::ALLGATHER_BASE);
    if (!o.is_same(out)) out.copy_(o);
    w.outputs_ = {out};
  });
}

std::shared_ptr<Work> HostRingPG::reduce_scatter_tensor(at::Tensor& output,
                                                        const at::Tensor& input, ReduceOp op) {
  RINGDP_CHECK(input.numel() == output.numel() * size_,
               "reduce_scatter_tensor: input numel must be world_size * output numel");
  at::Tensor out = output, in = input;
  return enqueue(coll_q_, OpType::REDUCE_SCATTER_BASE, [this, out, in, op](HostWork& w) mutable {
    at::Tensor buf = contig(in).clone();
    const int64_t per = out.numel();
    std::vector<int64_t> counts(size_, per), offs(size_);
    for (int i = 0; i < size_; ++i) offs[i] = per * i;
    if (size_ > 1)
      ring_reduce_scatter(static_cast<char*>(buf.data_ptr()), counts, offs, buf.scalar_type(),
                          buf.element_size(), op, w.seq(), OpType::REDUCE_SCATTER_BASE);
    at::Tensor mine = buf.view({-1}).narrow(0, per * rank_, per).view(out.sizes());
    if (op == ReduceOp::AVG) {
      mine = mine.clone();
      finish_avg(mine, size_);
    }
    out.copy_(mine);
    w.outputs_ = {out};
  });
}

std::shared_ptr<Work> HostRingPG::reduce(at::Tensor& tensor, int root, ReduceOp op) {
  at::Tensor t = tensor;
  return enqueue(coll_q_, OpType::REDUCE, [this, t, root, op](HostWork& w) mutable {
    at::Tensor c = contig(t).clone();
    ring_allreduce(c, op, w.seq());
    if (op == ReduceOp::AVG) finish_avg(c, size_);
    if (rank_ == root) t.copy_(c);
    w.outputs_ = {t};
  });
}

std::shared_ptr<Work> HostRingPG::gather(std::vector<at::Tensor>& outputs, const at::Tensor& input,
                                         int root) {
  auto outs = outputs;
  at::Tensor in = input;
  return enqueue(coll_q_, OpType::GATHER, [this, outs, in, root](HostWork& w) mutable {
    at::Tensor c = contig(in);
    if (rank_ == root) {
      RINGDP_CHECK(static_cast<int>(outs.size()) == size_, "gather: root needs world_size outputs");
      for (int i = 0; i < size_; ++i) {
        if (i == root) {
          outs[i].copy_(c);
          continue;
        }
        at::Tensor tmp = at::empty_like(c);
        recv_from(i, tmp.data_ptr(), tmp.nbytes(), w.seq(), OpType::GATHER, coll_fds_);
        outs[i].copy_(tmp);
      }
    } else {
      send_to(root, c.data_ptr(), c.nbytes(), w.seq(), OpType::GATHER, coll_fds_);
    }
    w.outputs_ = outs;
  });
}

std::shared_ptr<Work> HostRingPG::scatter(at::Tensor& output, std::vector<at::Tensor>& inputs,
                                          int root) {
  at::Tensor out = output;
  auto ins = inputs;
  return enqueue(coll_q_, OpType::SCATTER, [this, out, ins, root](HostWork& w) mutable {
    if (rank_ == root) {
      RINGDP_CHECK(static_cast<int>(ins.size()) == size_, "scatter: root needs world_size inputs");
      for (int i = 0; i < size_; ++i) {
        at::Tensor c = contig(ins[i]);
        if (i == root)
          out.copy_(c);
        else
          send_to(i, c.data_ptr(), c.nbytes(), w.seq(), OpType::SCATTER, coll_fds_);
      }
    } else {
      at::Tensor o = contig(out);
      recv_from(root, o.data_ptr(), o.nbytes(), w.seq(), OpType::SCATTER, coll_fds_);
      if (!o.is_same(out)) out.copy_(o);
    }
    w.outputs_ = {out};
  });
}

std::shared_ptr<Work> HostRingPG::alltoall_base(at::Tensor& output, const at::Tensor& input,
                                                const AllToAllSplits& splits) {
  at::Tensor out = output, in = input;
  AllToAllSplits sp = splits;
  return enqueue(coll_q_, OpType::ALLTOALL_BASE, [this, out, in, sp](HostWork& w) mutable {
    at::Tensor ci = contig(in);
    at::Tensor co = contig(out);
    const int n = size_;
    const int64_t row = ci.dim() > 0 ? ci.numel() / std::max<int64_t>(ci.size(0), 1) : 1;
    const size_t es = ci.element_size();
    std::vector<int64_t> isz(n), osz(n), ioff(n), ooff(n);
    for (int i = 0; i < n; ++i) {
      isz[i] = sp.input_split_sizes.empty() ? ci.size(0) / n : sp.input_split_sizes[i];
      osz[i] = sp.output_split_sizes.empty() ? co.size(0) / n : sp.output_split_sizes[i];
    }
    int64_t a = 0, b = 0;
    for (int i = 0; i < n; ++i) {
      ioff[i] = a;
      ooff[i] = b;
      a += isz[i];
      b += osz[i];
    }
    char* ip = static_cast<char*>(ci.data_ptr());
    char* op = static_cast<char*>(co.data_ptr());
    std::memcpy(op + ooff[rank_] * row * es, ip + ioff[rank_] * row * es, isz[rank_] * row * es);
    for (int k = 1; k < n; ++k) {
      int to = (rank_ + k) % n, from = (rank_ - k + n) % n;
      sendrecv(to, ip + ioff[to] * row * es, isz[to] * row * es, from,
               op + ooff[from] * row * es, osz[from] * row * es, w.seq(), OpType::ALLTOALL_BASE);
    }
    if (!co.is_same(out)) out.copy_(co);
    w.outputs_ = {out};
  });
}

std::shared_ptr<Work> HostRingPG::send(at::Tensor& tensor, int dst, int tag) {
  RINGDP_CHECK(dst >= 0 && dst < size_ && dst != rank_, "send: invalid dst ", dst);
  at::Tensor t = contig(tensor).clone();
  (void)tag;
  return enqueue(send_q_, OpType::SEND, [this, t, dst](HostWork& w) {
    send_to(dst, t.data_ptr(), t.nbytes(), w.seq(), OpType::SEND, p2p_fds_);
  });
}

std::shared_ptr<Work> HostRingPG::recv(at::Tensor& tensor, int src, int tag) {
  RINGDP_CHECK(src >= 0 && src < size_ && src != rank_, "recv: invalid src ", src);
  at::Tensor t = tensor;
  (void)tag;
  return enqueue(recv_q_, OpType::RECV, [this, t, src](HostWork& w) mutable {
    at::Tensor c = contig(t);
    recv_from(src, c.data_ptr(), c.nbytes(), w.seq(), OpType::SEND, p2p_fds_);
    if (!c.is_same(t)) t.copy_(c);
    w.outputs_ = {t};
  });
}

std::shared_ptr<Work> HostRingPG::barrier() {
  return enqueue(coll_q_, OpType::BARRIER, [this](HostWork& w) {
    at::Tensor t = at::ones({1}, at::kInt);
    // Reuse the ring; tag the messages as BARRIER for desync diagnostics.
    if (size_ > 1) {
      const int next = (rank_ + 1) % size_, prev = (rank_ + size_ - 1) % size_;
      int32_t token = 0;
      for (int s = 0; s < 2 * (size_ - 1); ++s)
        sendrecv(next, &token, sizeof(token), prev, &token, sizeof(token), w.seq(),
                 OpType::BARRIER);
    }
    (void)t;
  });
}

std::shared_ptr<ProcessGroup> HostRingPG::split(const std::vector<int>& ranks,
                                                const std::string& tag) {
  int new_rank = -1;
  for (size_t i = 0; i < ranks.size(); ++i)
    if (ranks[i] == rank_) new_rank = static_cast<int>(i);
  if (new_rank < 0) return nullptr;
  auto sub = std::make_shared<PrefixStore>(tag, store_);
  return std::make_shared<HostRingPG>(sub, new_rank, static_cast<int>(ranks.size()), timeout_,
                                      bind_hint_);
}

}  // namespace ringdp
