// HashStore (in-process) and FileStore (file:// rendezvous) implementations.
#include <fcntl.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <fstream>
#include <thread>

#include "store.h"
#include "wire.h"

namespace ringdp {

// ---------------------------------------------------------------- HashStore
void HashStore::set(const std::string& key, const std::string& value) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    data_[key] = value;
  }
  cv_.notify_all();
}

std::string HashStore::get(const std::string& key) {
  std::unique_lock<std::mutex> lk(mu_);
  if (!cv_.wait_for(lk, timeout_, [&] { return data_.count(key) > 0; }))
    throw TimeoutError(strcat_all("[ringdp] HashStore get('", key, "') timed out"));
  return data_[key];
}

int64_t HashStore::add(const std::string& key, int64_t delta) {
  int64_t v;
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = data_.find(key);
    v = (it == data_.end() || it->second.empty()) ? 0 : std::stoll(it->second);
    v += delta;
    data_[key] = std::to_string(v);
  }
  cv_.notify_all();
  return v;
}

std::string HashStore::compare_set(const std::string& key, const std::string& expected,
                                   const std::string& desired) {
  std::string out;
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = data_.find(key);
    if (it == data_.end()) {
      if (expected.empty()) {
        data_[key] = desired;
        out = desired;
      } else {
        out = expected;
      }
    } else if (it->second == expected) {
      it->second = desired;
      out = desired;
    } else {
      out = it->second;
    }
  }
  cv_.notify_all();
  return out;
}

bool HashStore::check(const std::vector<std::string>& keys) {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& k : keys)
    if (!data_.count(k)) return false;
  return true;
}

void HashStore::wait(const std::vector<std::string>& keys, std::chrono::milliseconds timeout) {
  std::unique_lock<std::mutex> lk(mu_);
  bool ok = cv_.wait_for(lk, timeout, [&] {
    for (auto& k : keys)
      if (!data_.count(k)) return false;
    return true;
  });
  if (!ok) throw TimeoutError("[ringdp] HashStore wait timed out");
}

bool HashStore::delete_key(const std::string& key) {
  std::lock_guard<std::mutex> lk(mu_);
  return data_.erase(key) > 0;
}

int64_t HashStore::num_keys() {
  std::lock_guard<std::mutex> lk(mu_);
  return static_cast<int64_t>(data_.size());
}

// ---------------------------------------------------------------- FileStore
// Log record: [u8 op (1=set, 2=delete)][str key][str value].
namespace {

struct FileLock {
  int fd;
  explicit FileLock(const std::string& path) {
    fd = ::open(path.c_str(), O_RDWR | O_CREAT, 0644);
    RINGDP_CHECK(fd >= 0, "FileStore: cannot open ", path, ": ", strerror(errno));
    while (::flock(fd, LOCK_EX) != 0) {
      RINGDP_CHECK(errno == EINTR, "FileStore: flock failed: ", strerror(errno));
    }
  }
  ~FileLock() {
    ::flock(fd, LOCK_UN);
    ::close(fd);
  }
  std::map<std::string, std::string> replay() {
    std::map<std::string, std::string> m;
    struct stat st{};
    ::fstat(fd, &st);
    std::string content(static_cast<size_t>(st.st_size), '\0');
    size_t off = 0;
    while (off < content.size()) {
      ssize_t r = ::pread(fd, content.data() + off, content.size() - off, off);
      if (r <= 0) break;
      off += static_cast<size_t>(r);
    }
    wire::Reader rd(content);
    while (rd.pos < content.size()) {
      uint8_t op = rd.u8();
      std::string k = rd.str();
      std::string v = rd.str();
      if (op == 1)
        m[k] = v;
      else
        m.erase(k);
    }
    return m;
  }
  void append(uint8_t op, const std::string& k, const std::string& v) {
    wire::Writer w;
    w.u8(op);
    w.str(k);
    w.str(v);
    ::lseek(fd, 0, SEEK_END);
    size_t off = 0;
    while (off < w.buf.size()) {
      ssize_t r = ::write(fd, w.buf.data() + off, w.buf.size() - off);
      RINGDP_CHECK(r > 0, "FileStore: write failed: ", strerror(errno));
      off += static_cast<size_t>(r);
    }
  }
};

}  // namespace

FileStore::FileStore(std::string path, int world_size, std::chrono::milliseconds timeout)
    : Store(timeout), path_(std::move(path)), world_size_(world_size) {
  FileLock lk(path_);  // create
}

FileStore::~FileStore() = default;

template <typename Fn>
auto FileStore::locked(Fn&& fn) {
  FileLock lk(path_);
  auto m = lk.replay();
  return fn(m, lk);
}

void FileStore::set(const std::string& key, const std::string& value) {
  locked([&](std::map<std::string, std::string>&, FileLock& lk) {
    lk.append(1, key, value);
    return 0;
  });
}

std::string FileStore::get(const std::string& key) {
  wait({key}, timeout_);
  return locked([&](std::map<std::string, std::string>& m, FileLock&) { return m.at(key); });
}

int64_t FileStore::add(const std::string& key, int64_t delta) {
  return locked([&](std::map<std::string, std::string>& m, FileLock& lk) {
    auto it = m.find(key);
    int64_t v = (it == m.end() || it->second.empty()) ? 0 : std::stoll(it->second);
    v += delta;
    lk.append(1, key, std::to_string(v));
    return v;
  });
}

std::string FileStore::compare_set(const std::string& key, const std::string& expected,
                                   const std::string& desired) {
  return locked([&](std::map<std::string, std::string>& m, FileLock& lk) {
    auto it = m.find(key);
    if (it == m.end()) {
      if (expected.empty()) {
        lk.append(1, key, desired);
        return desired;
      }
      return expected;
    }
    if (it->second == expected) {
      lk.append(1, key, desired);
      return desired;
    }
    return it->second;
  });
}

bool FileStore::check(const std::vector<std::string>& keys) {
  return locked([&](std::map<std::string, std::string>& m, FileLock&) {
    for (auto& k : keys)
      if (!m.count(k)) return false;
    return true;
  });
}

void FileStore::wait(const std::vector<std::string>& keys, std::chrono::milliseconds timeout) {
  auto deadline = Clock::now() + timeout;
  int sleep_ms = 1;
  while (!check(keys)) {
    if (Clock::now() > deadline) throw TimeoutError("[ringdp] FileStore wait timed out");
    std::this_thread::sleep_for(std::chrono::milliseconds(sleep_ms));
    sleep_ms = std::min(sleep_ms * 2, 50);
  }
}

bool FileStore::delete_key(const std::string& key) {
  return locked([&](std::map<std::string, std::string>& m, FileLock& lk) {
    if (!m.count(key)) return false;
    lk.append(2, key, "");
    return true;
  });
}

int64_t FileStore::num_keys() {
  return locked([&](std::map<std::string, std::string>& m, FileLock&) {
    return static_cast<int64_t>(m.size());
  });
}

}  // namespace ringdp
