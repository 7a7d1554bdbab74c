// ringdp key-value stores used for rendezvous / bootstrap (unique-id exchange, barriers).
//
// Parity target: the c10d Store family the reference reaches through
// `init_process_group(init_method='env://'|'tcp://')` (SURVEY.md §2.3 U2/U3,
// torch/distributed/rendezvous.py:163-208, c10d/TCPStore.hpp:73).  Semantics kept:
// blocking get/wait with a timeout, integer `add` stored as decimal text,
// compare_set, check, delete, num_keys, and key prefixing per process group.
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../common.h"

namespace ringdp {

class Store {
 public:
  explicit Store(std::chrono::milliseconds timeout) : timeout_(timeout) {}
  virtual ~Store() = default;

  virtual void set(const std::string& key, const std::string& value) = 0;
  // Blocks until `key` exists or the store timeout expires.
  virtual std::string get(const std::string& key) = 0;
  virtual int64_t add(const std::string& key, int64_t delta) = 0;
  // Returns the value after the operation (desired when swapped, the current value otherwise;
  // `expected` when the key is missing and expected != "" ... mirrors c10d).
  virtual std::string compare_set(const std::string& key, const std::string& expected,
                                  const std::string& desired) = 0;
  virtual bool check(const std::vector<std::string>& keys) = 0;
  virtual void wait(const std::vector<std::string>& keys, std::chrono::milliseconds timeout) = 0;
  void wait(const std::vector<std::string>& keys) { wait(keys, timeout_); }
  virtual bool delete_key(const std::string& key) = 0;
  virtual int64_t num_keys() = 0;

  std::chrono::milliseconds timeout() const { return timeout_; }
  void set_timeout(std::chrono::milliseconds t) { timeout_ = t; }

 protected:
  std::chrono::milliseconds timeout_;
};

// In-process store (single process, multi-thread); used by tests and world_size==1.
class HashStore : public Store {
 public:
  explicit HashStore(std::chrono::milliseconds timeout) : Store(timeout) {}
  void set(const std::string& key, const std::string& value) override;
  std::string get(const std::string& key) override;
  int64_t add(const std::string& key, int64_t delta) override;
  std::string compare_set(const std::string& key, const std::string& expected,
                          const std::string& desired) override;
  bool check(const std::vector<std::string>& keys) override;
  void wait(const std::vector<std::string>& keys, std::chrono::milliseconds timeout) override;
  bool delete_key(const std::string& key) override;
  int64_t num_keys() override;

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, std::string> data_;
};

class PrefixStore : public Store {
 public:
  PrefixStore(std::string prefix, std::shared_ptr<Store> base)
      : Store(base->timeout()), prefix_(std::move(prefix)), base_(std::move(base)) {}
  void set(const std::string& key, const std::string& value) override {
    base_->set(k(key), value);
  }
  std::string get(const std::string& key) override { return base_->get(k(key)); }
  int64_t add(const std::string& key, int64_t delta) override { return base_->add(k(key), delta); }
  std::string compare_set(const std::string& key, const std::string& expected,
                          const std::string& desired) override {
    return base_->compare_set(k(key), expected, desired);
  }
  bool check(const std::vector<std::string>& keys) override { return base_->check(ks(keys)); }
  void wait(const std::vector<std::string>& keys, std::chrono::milliseconds timeout) override {
    base_->wait(ks(keys), timeout);
  }
  bool delete_key(const std::string& key) override { return base_->delete_key(k(key)); }
  int64_t num_keys() override { return base_->num_keys(); }
  std::shared_ptr<Store> underlying() const { return base_; }
  const std::string& prefix() const { return prefix_; }

 private:
  std::string k(const std::string& key) const { return prefix_ + "/" + key; }
  std::vector<std::string> ks(const std::vector<std::string>& keys) const {
    std::vector<std::string> out;
    out.reserve(keys.size());
    for (auto& key : keys) out.push_back(k(key));
    return out;
  }
  std::string prefix_;
  std::shared_ptr<Store> base_;
};

class TCPStoreServer;

// TCP store: rank 0 (is_master) hosts a poll()-driven server thread; every rank is a client.
class TCPStore : public Store {
 public:
  TCPStore(const std::string& host, int port, bool is_master, std::chrono::milliseconds timeout,
           int world_size = -1, bool wait_for_workers = false);
  ~TCPStore() override;

  void set(const std::string& key, const std::string& value) override;
  std::string get(const std::string& key) override;
  int64_t add(const std::string& key, int64_t delta) override;
  std::string compare_set(const std::string& key, const std::string& expected,
                          const std::string& desired) override;
  bool check(const std::vector<std::string>& keys) override;
  void wait(const std::vector<std::string>& keys, std::chrono::milliseconds timeout) override;
  bool delete_key(const std::string& key) override;
  int64_t num_keys() override;

  int port() const { return port_; }
  const std::string& host() const { return host_; }
  bool is_master() const { return server_ != nullptr; }

 private:
  std::string request(const std::string& payload, std::chrono::milliseconds timeout);
  std::string host_;
  int port_;
  int fd_ = -1;
  std::mutex mu_;
  std::unique_ptr<TCPStoreServer> server_;
};

// File-backed store (init_method='file://path'): an append-only record log guarded by flock.
class FileStore : public Store {
 public:
  FileStore(std::string path, int world_size, std::chrono::milliseconds timeout);
  ~FileStore() override;
  void set(const std::string& key, const std::string& value) override;
  std::string get(const std::string& key) override;
  int64_t add(const std::string& key, int64_t delta) override;
  std::string compare_set(const std::string& key, const std::string& expected,
                          const std::string& desired) override;
  bool check(const std::vector<std::string>& keys) override;
  void wait(const std::vector<std::string>& keys, std::chrono::milliseconds timeout) override;
  bool delete_key(const std::string& key) override;
  int64_t num_keys() override;

 private:
  // Runs `fn(map)` under an exclusive lock after replaying the log; appends any records fn emits.
  template <typename Fn>
  auto locked(Fn&& fn);
  std::string path_;
  int world_size_;
};

}  // namespace ringdp
