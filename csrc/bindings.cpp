// pybind11 module `ringdp._C`: stores, process groups, reducer, HIP ops.
#include <torch/extension.h>
#include <pybind11/chrono.h>
#include <pybind11/functional.h>
#include <pybind11/stl.h>

#include "comm/fake_pg.h"
#include "comm/host_ring.h"
#include "comm/rccl_pg.h"
#include "comm/xgmi_pg.h"
#include "ops/nn_ops.h"
#include "ops/ops.h"
#include "reducer/reducer.h"
#include "store/store.h"
#include "trace/trace.h"

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <thread>

namespace py = pybind11;
using namespace ringdp;

namespace {

std::chrono::milliseconds ms(int64_t v) { return std::chrono::milliseconds(v); }

py::bytes to_bytes(const std::string& s) { return py::bytes(s); }

std::string as_str(const py::object& o) {
  if (py::isinstance<py::bytes>(o)) return o.cast<std::string>();
  if (py::isinstance<py::str>(o)) return o.cast<std::string>();
  return py::str(o).cast<std::string>();
}

// A Store backed by any Python object exposing set/get/add/wait/check/delete_key/num_keys/
// compare_set (e.g. torch.distributed.TCPStore when ringdp workers are started by torchrun and
// must rendezvous through the elastic agent's store instead of hosting their own).
class PyStore : public Store {
 public:
  PyStore(py::object obj, std::chrono::milliseconds timeout) : Store(timeout), obj_(std::move(obj)) {}
  ~PyStore() override {
    py::gil_scoped_acquire gil;
    obj_ = py::object();
  }
  void set(const std::string& key, const std::string& value) override {
    py::gil_scoped_acquire gil;
    obj_.attr("set")(key, py::bytes(value));
  }
  std::string get(const std::string& key) override {
    py::gil_scoped_acquire gil;
    return obj_.attr("get")(key).cast<std::string>();
  }
  int64_t add(const std::string& key, int64_t delta) override {
    py::gil_scoped_acquire gil;
    return obj_.attr("add")(key, delta).cast<int64_t>();
  }
  std::string compare_set(const std::string& key, const std::string& expected,
                          const std::string& desired) override {
    py::gil_scoped_acquire gil;
    return obj_.attr("compare_set")(key, py::bytes(expected), py::bytes(desired)).cast<std::string>();
  }
  bool check(const std::vector<std::string>& keys) override {
    py::gil_scoped_acquire gil;
    return obj_.attr("check")(keys).cast<bool>();
  }
  void wait(const std::vector<std::string>& keys, std::chrono::milliseconds timeout) override {
    py::gil_scoped_acquire gil;
    obj_.attr("wait")(keys, timeout);
  }
  bool delete_key(const std::string& key) override {
    py::gil_scoped_acquire gil;
    return obj_.attr("delete_key")(key).cast<bool>();
  }
  int64_t num_keys() override {
    py::gil_scoped_acquire gil;
    return obj_.attr("num_keys")().cast<int64_t>();
  }

 private:
  py::object obj_;
};

// Adapts a Python object with wait()/result() (e.g. a comm-hook future) to a native Work.
class PyWork : public Work {
 public:
  explicit PyWork(py::object obj) : Work(OpType::COALESCED, 0), obj_(std::move(obj)) {}
  ~PyWork() override {
    py::gil_scoped_acquire gil;
    obj_ = py::object();
  }
  void wait(bool /*blocking*/) override {
    py::gil_scoped_acquire gil;
    py::object r = obj_.attr("wait")();
    if (py::hasattr(obj_, "result")) {
      py::object res = obj_.attr("result")();
      if (py::isinstance<at::Tensor>(res)) {
        outputs_ = {res.cast<at::Tensor>()};
      } else {
        try {
          outputs_ = res.cast<std::vector<at::Tensor>>();
        } catch (const py::cast_error&) {
        }
      }
    } else if (py::isinstance<at::Tensor>(r)) {
      outputs_ = {r.cast<at::Tensor>()};
    }
  }
  bool is_completed() override {
    py::gil_scoped_acquire gil;
    if (py::hasattr(obj_, "is_completed")) return obj_.attr("is_completed")().cast<bool>();
    if (py::hasattr(obj_, "done")) return obj_.attr("done")().cast<bool>();
    return false;
  }

 private:
  py::object obj_;
};

}  // namespace

namespace {
// RINGDP_ABORT_BACKTRACE=1: a SIGABRT (std::terminate, failed asserts) prints the native stack to stderr before
// the default action - diagnosis of aborts that happen outside any Python frame (e.g. at process teardown).
void abort_backtrace(int sig) {
  static const char kMsg[] = "[ringdp] SIGABRT, native stack:\n";
  (void)!::write(2, kMsg, sizeof(kMsg) - 1);
  void* frames[64];
  const int n = ::backtrace(frames, 64);
  ::backtrace_symbols_fd(frames, n, 2);
  ::signal(sig, SIG_DFL);
  ::raise(sig);
}
}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  if (const char* e = std::getenv("RINGDP_ABORT_BACKTRACE"); e && *e && *e != '0') ::signal(SIGABRT, abort_backtrace);
  m.doc() = "ringdp native runtime for AMD MI355X (gfx950): stores, RCCL/host-ring process "
            "groups, gradient reducer and CDNA4 HIP kernels";

  py::register_exception<RingdpError>(m, "RingdpError", PyExc_RuntimeError);
  py::register_exception<TimeoutError>(m, "DistTimeoutError", PyExc_TimeoutError);

  // ---------------------------------------------------------------- stores
  py::class_<Store, std::shared_ptr<Store>>(m, "Store")
      .def("set", [](Store& s, const std::string& k, const py::object& v) { s.set(k, as_str(v)); })
      .def("get",
           [](Store& s, const std::string& k) {
             std::string v;
             {
               py::gil_scoped_release nogil;
               v = s.get(k);
             }
             return to_bytes(v);
           })
      .def("add", &Store::add, py::call_guard<py::gil_scoped_release>())
      .def("compare_set",
           [](Store& s, const std::string& k, const py::object& e, const py::object& d) {
             std::string es = as_str(e), ds = as_str(d), v;
             {
               py::gil_scoped_release nogil;
               v = s.compare_set(k, es, ds);
             }
             return to_bytes(v);
           })
      .def("check", &Store::check, py::call_guard<py::gil_scoped_release>())
      .def("wait",
           [](Store& s, const std::vector<std::string>& keys) {
             py::gil_scoped_release nogil;
             s.wait(keys);
           })
      .def("wait",
           [](Store& s, const std::vector<std::string>& keys, const std::chrono::milliseconds& t) {
             py::gil_scoped_release nogil;
             s.wait(keys, t);
           })
      .def("delete_key", &Store::delete_key, py::call_guard<py::gil_scoped_release>())
      .def("num_keys", &Store::num_keys, py::call_guard<py::gil_scoped_release>())
      .def_property("timeout", &Store::timeout, &Store::set_timeout)
      .def("set_timeout", &Store::set_timeout);

  py::class_<HashStore, Store, std::shared_ptr<HashStore>>(m, "HashStore")
      .def(py::init([](int64_t timeout_ms) { return std::make_shared<HashStore>(ms(timeout_ms)); }),
           py::arg("timeout_ms") = 300000);

  py::class_<PrefixStore, Store, std::shared_ptr<PrefixStore>>(m, "PrefixStore")
      .def(py::init([](const std::string& prefix, std::shared_ptr<Store> base) {
             return std::make_shared<PrefixStore>(prefix, std::move(base));
           }),
           py::arg("prefix"), py::arg("store"))
      .def_property_readonly("underlying_store", &PrefixStore::underlying)
      .def_property_readonly("prefix", &PrefixStore::prefix);

  py::class_<TCPStore, Store, std::shared_ptr<TCPStore>>(m, "TCPStore")
      .def(py::init([](const std::string& host, int port, int world_size, bool is_master,
                       int64_t timeout_ms, bool wait_for_workers) {
             py::gil_scoped_release nogil;
             return std::make_shared<TCPStore>(host, port, is_master, ms(timeout_ms), world_size,
                                               wait_for_workers);
           }),
           py::arg("host_name"), py::arg("port"), py::arg("world_size") = -1,
           py::arg("is_master") = false, py::arg("timeout_ms") = 300000,
           py::arg("wait_for_workers") = false)
      .def_property_readonly("port", &TCPStore::port)
      .def_property_readonly("host", &TCPStore::host)
      .def_property_readonly("is_master", &TCPStore::is_master);

  py::class_<FileStore, Store, std::shared_ptr<FileStore>>(m, "FileStore")
      .def(py::init([](const std::string& path, int world_size, int64_t timeout_ms) {
             return std::make_shared<FileStore>(path, world_size, ms(timeout_ms));
           }),
           py::arg("path"), py::arg("world_size") = -1, py::arg("timeout_ms") = 300000);

  py::class_<PyStore, Store, std::shared_ptr<PyStore>>(m, "PyStore")
      .def(py::init([](py::object obj, int64_t timeout_ms) {
             return std::make_shared<PyStore>(std::move(obj), ms(timeout_ms));
           }),
           py::arg("store"), py::arg("timeout_ms") = 300000);

  // ---------------------------------------------------------------- process groups
  py::enum_<ReduceOp>(m, "ReduceOp")
      .value("SUM", ReduceOp::SUM)
      .value("PRODUCT", ReduceOp::PRODUCT)
      .value("MIN", ReduceOp::MIN)
      .value("MAX", ReduceOp::MAX)
      .value("AVG", ReduceOp::AVG)
      .value("BAND", ReduceOp::BAND)
      .value("BOR", ReduceOp::BOR)
      .value("BXOR", ReduceOp::BXOR);

  py::class_<Work, std::shared_ptr<Work>>(m, "Work")
      .def("wait",
           [](Work& w, bool blocking) {
             py::gil_scoped_release nogil;
             w.wait(blocking);
             return true;
           },
           py::arg("blocking") = false)
      .def("is_completed", &Work::is_completed)
      .def("synchronize", &Work::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("result", [](Work& w) { return w.result(); })
      .def_property_readonly("seq", &Work::seq)
      .def_property_readonly("op", [](Work& w) { return std::string(op_name(w.op())); })
      .def("duration_us", &Work::duration_us);

  py::class_<ProcessGroup, std::shared_ptr<ProcessGroup>>(m, "ProcessGroup")
      .def("rank", &ProcessGroup::rank)
      .def("size", &ProcessGroup::size)
      .def("backend_name", &ProcessGroup::backend_name)
      .def("seq", &ProcessGroup::seq)
      .def("allreduce", &ProcessGroup::allreduce, py::call_guard<py::gil_scoped_release>())
      .def("allreduce_coalesced", &ProcessGroup::allreduce_coalesced,
           py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &ProcessGroup::broadcast, py::call_guard<py::gil_scoped_release>())
      .def("allgather", &ProcessGroup::allgather, py::call_guard<py::gil_scoped_release>())
      .def("allgather_into_tensor", &ProcessGroup::allgather_into_tensor,
           py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter_tensor", &ProcessGroup::reduce_scatter_tensor,
           py::call_guard<py::gil_scoped_release>())
      .def("reduce", &ProcessGroup::reduce, py::call_guard<py::gil_scoped_release>())
      .def("gather", &ProcessGroup::gather, py::call_guard<py::gil_scoped_release>())
      .def("scatter", &ProcessGroup::scatter, py::call_guard<py::gil_scoped_release>())
      .def("alltoall_base",
           [](ProcessGroup& pg, at::Tensor& out, const at::Tensor& in,
              std::vector<int64_t> out_splits, std::vector<int64_t> in_splits) {
             py::gil_scoped_release nogil;
             AllToAllSplits sp{std::move(out_splits), std::move(in_splits)};
             return pg.alltoall_base(out, in, sp);
           })
      .def("send", &ProcessGroup::send, py::call_guard<py::gil_scoped_release>())
      .def("recv", &ProcessGroup::recv, py::call_guard<py::gil_scoped_release>())
      .def("barrier", &ProcessGroup::barrier, py::call_guard<py::gil_scoped_release>())
      .def("split", &ProcessGroup::split, py::call_guard<py::gil_scoped_release>())
      .def("coalesced",
           [](ProcessGroup& pg, const std::vector<py::tuple>& items) {
             // items: (kind, out, in_or_None, root, ReduceOp)
             std::vector<CollOp> ops;
             for (auto& it : items) {
               CollOp c;
               c.kind = it[0].cast<int>();
               c.out = it[1].cast<at::Tensor>();
               if (!it[2].is_none()) c.in = it[2].cast<at::Tensor>();
               c.root = it[3].cast<int>();
               c.op = it[4].cast<ReduceOp>();
               ops.push_back(std::move(c));
             }
             py::gil_scoped_release nogil;
             return pg.coalesced(ops);
           })
      .def("shutdown", &ProcessGroup::shutdown, py::call_guard<py::gil_scoped_release>())
      .def("abort", &ProcessGroup::abort, py::call_guard<py::gil_scoped_release>());

  py::class_<FakePG, ProcessGroup, std::shared_ptr<FakePG>>(m, "FakePG")
      .def(py::init<int, int>(), py::arg("rank"), py::arg("size"));

  py::class_<HostRingPG, ProcessGroup, std::shared_ptr<HostRingPG>>(m, "HostRingPG")
      .def(py::init([](std::shared_ptr<Store> store, int rank, int size, int64_t timeout_ms,
                       const std::string& bind_hint) {
             py::gil_scoped_release nogil;
             return std::make_shared<HostRingPG>(std::move(store), rank, size, ms(timeout_ms),
                                                 bind_hint);
           }),
           py::arg("store"), py::arg("rank"), py::arg("size"), py::arg("timeout_ms") = 1800000,
           py::arg("bind_hint") = "127.0.0.1");

  py::class_<ReplayBeacon, std::shared_ptr<ReplayBeacon>>(m, "ReplayBeacon")
      .def(py::init<int>(), py::arg("device"))
      .def("mark", [](ReplayBeacon& b, uint64_t stream) { b.mark(reinterpret_cast<hipStream_t>(stream)); },
           py::arg("stream"), "enqueue the completion marker (inside the capture, after the step)")
      .def("issued", &ReplayBeacon::issued)
      .def("issued_count", &ReplayBeacon::issued_count)
      .def("completed", &ReplayBeacon::completed)
      .def_property_readonly("device", &ReplayBeacon::device);
  py::class_<GpuPG, ProcessGroup, std::shared_ptr<GpuPG>>(m, "GpuPG")
      .def_property_readonly("device", &GpuPG::device)
      .def("aborted", &GpuPG::aborted)
      .def("drain", &GpuPG::drain, py::call_guard<py::gil_scoped_release>())
      .def("error_message", &GpuPG::error_message)
      .def("set_timing", &GpuPG::set_timing)
      .def("timing", &GpuPG::timing)
      .def("same_stream", &GpuPG::same_stream)
      .def("set_same_stream", &GpuPG::set_same_stream, py::call_guard<py::gil_scoped_release>())
      .def("watch_beacon", &GpuPG::watch_beacon, py::arg("beacon"),
           "watchdog-track the replays of a captured step through its ReplayBeacon")
      .def("join_into",
           [](GpuPG& pg, uint64_t stream) { pg.join_into(reinterpret_cast<hipStream_t>(stream)); },
           py::arg("stream"), "make `stream` wait for the last eager op of this group")
      .def("set_async_error_handling", &GpuPG::set_async_error_handling)
      .def("backend_failure", &GpuPG::backend_failure)
      .def("comm_stream_ptr", [](GpuPG& pg) { return reinterpret_cast<uintptr_t>(pg.comm_stream()); });
  py::class_<RcclPG, GpuPG, std::shared_ptr<RcclPG>>(m, "RcclPG")
      .def(py::init([](std::shared_ptr<Store> store, int rank, int size, int device,
                       int64_t timeout_ms) {
             py::gil_scoped_release nogil;
             return std::make_shared<RcclPG>(std::move(store), rank, size, device, ms(timeout_ms));
           }),
           py::arg("store"), py::arg("rank"), py::arg("size"), py::arg("device"),
           py::arg("timeout_ms") = 600000)
      .def("p2p_max_bytes", &RcclPG::p2p_max_bytes)
      .def("set_p2p_enabled", &RcclPG::set_p2p_enabled)
      .def("split_with_timeout", &RcclPG::split_with_timeout, py::arg("ranks"), py::arg("tag"),
           py::arg("timeout_ms"), py::call_guard<py::gil_scoped_release>());
  // Own-kernel collectives over IPC-mapped peer memory: one node, ranks may share a GPU.
  py::class_<XgmiPG, GpuPG, std::shared_ptr<XgmiPG>>(m, "XgmiPG")
      .def(py::init([](std::shared_ptr<Store> store, int rank, int size, int device,
                       int64_t timeout_ms) {
             py::gil_scoped_release nogil;
             return std::make_shared<XgmiPG>(std::move(store), rank, size, device, ms(timeout_ms));
           }),
           py::arg("store"), py::arg("rank"), py::arg("size"), py::arg("device"),
           py::arg("timeout_ms") = 600000)
      .def("config", [](XgmiPG& pg) {
        const auto& c = pg.config();
        py::dict d;
        d["nblocks"] = c.nblocks;
        d["slot_bytes"] = c.slot_bytes;
        d["p2p_slot_bytes"] = c.p2p_slot_bytes;
        d["oneshot_max"] = c.oneshot_max;
        return d;
      });

  // Exit guard (bench.py): a native thread that, unless cancelled within `seconds`, writes `text` to
  // stdout and ends the process with status 3 (a hang is never reported as success; the launcher
  // and CI see the failure).  Native, so it fires even while the main thread is stuck inside a call
  // that holds the GIL.
  {
    struct Guard {
      std::mutex mu;
      std::condition_variable cv;
      bool cancelled = false;
    };
    static std::shared_ptr<Guard> guard;
    m.def(
        "exit_guard_arm",
        [](double seconds, std::string text) {
          auto g = std::make_shared<Guard>();
          guard = g;
          std::thread([g, seconds, text = std::move(text)] {
            std::unique_lock<std::mutex> lk(g->mu);
            if (g->cv.wait_for(lk, std::chrono::duration<double>(seconds), [&] { return g->cancelled; })) return;
            if (!text.empty()) {
              ssize_t off = 0;
              while (off < (ssize_t)text.size()) {
                const ssize_t n = ::write(1, text.data() + off, text.size() - off);
                if (n <= 0) break;
                off += n;
              }
            }
            static const char kMsg[] = "[ringdp] exit guard fired: a phase stopped making progress; exiting with status 3\n";
            (void)!::write(2, kMsg, sizeof(kMsg) - 1);
            std::fflush(stderr);
            std::_Exit(3);
          }).detach();
        },
        py::arg("seconds"), py::arg("text"));
    m.def("exit_guard_cancel", []() {
      if (!guard) return;
      {
        std::lock_guard<std::mutex> lk(guard->mu);
        guard->cancelled = true;
      }
      guard->cv.notify_all();
      guard.reset();
    });
  }

  m.def("rccl_version", []() {
    int v = 0;
    ncclGetVersion(&v);
    return v;
  });

  // ---------------------------------------------------------------- reducer
  py::enum_<CommHook>(m, "CommHook")
      .value("ALLREDUCE", CommHook::ALLREDUCE)
      .value("BF16_COMPRESS", CommHook::BF16_COMPRESS)
      .value("FP16_COMPRESS", CommHook::FP16_COMPRESS)
      .value("PYTHON", CommHook::PYTHON)
      .value("NONE", CommHook::NONE);

  py::class_<BucketStats>(m, "BucketStats")
      .def_readonly("numel", &BucketStats::numel)
      .def_readonly("bytes", &BucketStats::bytes)
      .def_readonly("last_ready_us", &BucketStats::last_ready_us)
      .def_readonly("last_launch_us", &BucketStats::last_launch_us)
      .def_readonly("last_comm_us", &BucketStats::last_comm_us)
      .def_readonly("total_comm_us", &BucketStats::total_comm_us)
      .def_readonly("comm_samples", &BucketStats::comm_samples);

  py::class_<Reducer, std::shared_ptr<Reducer>>(m, "Reducer")
      .def(py::init<std::vector<at::Tensor>, std::vector<std::vector<int64_t>>,
                    std::shared_ptr<ProcessGroup>, bool, int64_t>(),
           py::arg("params"), py::arg("bucket_indices"), py::arg("process_group"),
           py::arg("find_unused_parameters") = false, py::arg("pad_elems") = 16)
      .def("prepare_for_forward", &Reducer::prepare_for_forward)
      .def("prepare_for_backward", &Reducer::prepare_for_backward)
      .def("set_require_sync", &Reducer::set_require_sync)
      .def("require_sync", &Reducer::require_sync)
      .def("set_comm_hook", &Reducer::set_comm_hook)
      .def("comm_hook", &Reducer::comm_hook)
      .def("set_python_hook",
           [](Reducer& r, py::function fn) {
             auto holder = std::make_shared<py::function>(std::move(fn));
             r.set_python_hook([holder](int64_t idx, at::Tensor flat) -> std::shared_ptr<Work> {
               py::gil_scoped_acquire gil;
               py::object res = (*holder)(idx, flat);
               if (res.is_none()) return nullptr;
               if (py::isinstance<Work>(res)) return res.cast<std::shared_ptr<Work>>();
               return std::make_shared<PyWork>(res);
             });
           })
      .def("set_capture_split",
           [](Reducer& r, py::object fn) {
             if (fn.is_none()) {
               r.set_capture_split(nullptr);
               return;
             }
             auto holder = std::shared_ptr<py::function>(new py::function(fn.cast<py::function>()),
                                                         [](py::function* f) {
                                                           py::gil_scoped_acquire gil;
                                                           delete f;
                                                         });
             r.set_capture_split([holder](int64_t idx) -> bool {
               py::gil_scoped_acquire gil;
               return (*holder)(idx).cast<bool>();
             });
           })
      .def("launch_collective", &Reducer::launch_collective, py::call_guard<py::gil_scoped_release>())
      .def("grad_slots", &Reducer::grad_slots)
      .def("flat_buffers", &Reducer::flat_buffers)
      .def("param_offsets", &Reducer::param_offsets)
      .def("bucket_indices", &Reducer::bucket_indices)
      .def("bucket_numels", &Reducer::bucket_numels)
      .def("ready_order", &Reducer::ready_order)
      .def("rebuilt", &Reducer::rebuilt)
      .def("rebuild_buckets", &Reducer::rebuild_buckets)
      .def("iteration", &Reducer::iteration)
      .def("stats", &Reducer::stats)
      .def("collect_comm_times", &Reducer::collect_comm_times);

  m.def("compute_bucket_assignment_by_size",
        [](const std::vector<at::Tensor>& tensors, const std::vector<int64_t>& limits,
           const std::vector<bool>& expect_sparse, const std::vector<int64_t>& tensor_indices) {
          return compute_bucket_assignment_by_size(tensors, limits, expect_sparse, tensor_indices);
        },
        py::arg("tensors"), py::arg("bucket_size_limits"),
        py::arg("expect_sparse_gradient") = std::vector<bool>{},
        py::arg("tensor_indices") = std::vector<int64_t>{});

  // ---------------------------------------------------------------- ops
  py::class_<ops::SgdHyper>(m, "SgdHyper")
      .def(py::init<>())
      .def_readwrite("lr", &ops::SgdHyper::lr)
      .def_readwrite("momentum", &ops::SgdHyper::momentum)
      .def_readwrite("dampening", &ops::SgdHyper::dampening)
      .def_readwrite("weight_decay", &ops::SgdHyper::weight_decay)
      .def_readwrite("nesterov", &ops::SgdHyper::nesterov)
      .def_readwrite("maximize", &ops::SgdHyper::maximize);
  m.def("cast_copy", &ops::cast_copy);
  m.def("cast_bf16_multi", &ops::cast_bf16_multi);
  m.def("cast_bf16_t_multi", &ops::cast_bf16_t_multi);
  m.def("transpose_bf16", &ops::transpose_bf16);
  m.def("sgd_flat", &ops::sgd_flat, py::arg("param"), py::arg("grad"), py::arg("momentum_buf"),
        py::arg("hyper"), py::arg("first_step"), py::arg("lr_tensor") = py::none(),
        py::arg("grad_scale") = py::none(), py::arg("packed") = py::none(),
        py::arg("pack_offsets") = std::vector<int64_t>{});
  m.def("sgd_multi", &ops::sgd_multi, py::arg("params"), py::arg("grads"), py::arg("bufs"),
        py::arg("hyper"), py::arg("first_step"), py::arg("lr_tensor") = py::none(),
        py::arg("grad_scale") = py::none());
  m.def("sgd_multi_build", &ops::sgd_multi_build);
  m.def("sgd_multi_run", &ops::sgd_multi_run, py::arg("table"), py::arg("nchunks"),
        py::arg("table_bytes"), py::arg("hyper"), py::arg("first_step"),
        py::arg("lr_tensor") = py::none(), py::arg("grad_scale") = py::none());
  m.def("cross_entropy_fwd", &ops::cross_entropy_fwd);
  m.def("cross_entropy_bwd", &ops::cross_entropy_bwd);
  // roctx tracing (rocprofv3 --marker-trace)
  m.def("trace_enabled", &trace::enabled);
  m.def("trace_set_enabled", &trace::set_enabled);
  m.def("trace_push", [](const std::string& n) { trace::push(n.c_str()); });
  m.def("trace_pop", &trace::pop);
  m.def("trace_mark", [](const std::string& n) { trace::mark(n.c_str()); });
  m.def("gather_augment", &ops::gather_augment, py::arg("x"), py::arg("labels"), py::arg("idx"),
        py::arg("pad") = 0, py::arg("flip") = false, py::arg("mean") = std::vector<double>{},
        py::arg("std") = std::vector<double>{}, py::arg("seed") = 0, py::arg("nhwc") = false,
        py::arg("out_dtype") = at::kFloat);
  // generic GEMM / implicit-GEMM conv / NHWC layers
  m.def("gemm", &ops::gemm, py::arg("a"), py::arg("b"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("lda"),
        py::arg("ldb"), py::arg("a_row") = false, py::arg("b_row") = false, py::arg("batch") = 1,
        py::arg("a_bstride") = 0, py::arg("b_bstride") = 0, py::arg("out_bf16") = true,
        py::arg("bias") = py::none(), py::arg("act") = 0, py::arg("residual") = py::none(),
        py::arg("preact") = py::none(), py::arg("alpha") = 1.0, py::arg("out") = py::none(),
        py::arg("colsum") = py::none());
  m.def("gemm_splitk_f32", &ops::gemm_splitk_f32);
  m.def("pack_conv_weight", &ops::pack_conv_weight);
  m.def("pack_conv_weights", &ops::pack_conv_weights);
  m.def("conv2d_fwd", &ops::conv2d_fwd);
  m.def("conv2d_dgrad", &ops::conv2d_dgrad, py::arg("dz"), py::arg("w_crsk"), py::arg("H"), py::arg("W"),
        py::arg("stride"), py::arg("pad"), py::arg("dil"), py::arg("residual") = py::none());
  m.def("conv2d_wgrad", &ops::conv2d_wgrad);
  m.def("nchw_to_nhwc", &ops::nchw_to_nhwc);
  m.def("bn_fwd_train", &ops::bn_fwd_train, py::arg("z"), py::arg("sums"), py::arg("gamma"), py::arg("beta"),
        py::arg("running_mean"), py::arg("running_var"), py::arg("eps"), py::arg("momentum"), py::arg("residual"),
        py::arg("relu"), py::arg("num_batches_tracked") = py::none());
  m.def("bn_fwd_eval", &ops::bn_fwd_eval);
  m.def("bn_bwd", &ops::bn_bwd, py::arg("dy"), py::arg("y"), py::arg("z"), py::arg("save"), py::arg("gamma"),
        py::arg("relu"), py::arg("dgamma"), py::arg("dbeta"), py::arg("need_g") = true);
  m.def("maxpool2d_fwd", &ops::maxpool2d_fwd);
  m.def("maxpool2d_bwd", &ops::maxpool2d_bwd);
  m.def("avgpool_fwd", &ops::avgpool_fwd);
  m.def("avgpool_bwd", &ops::avgpool_bwd);
  m.def("head_ok", [](int64_t C, int64_t J) { return kern::head_ok((int)C, (int)J); });
  m.def("head_fwd", &ops::head_fwd);
  m.def("head_bwd", &ops::head_bwd);
  m.def("add_bf16", &ops::add_bf16);
  m.def("layernorm_fwd", &ops::layernorm_fwd);
  m.def("layernorm_bwd", &ops::layernorm_bwd);
  m.def("layernorm_fwd_q8", &ops::layernorm_fwd_q8, "layernorm forward with e4m3 outputs (q, q^T) at a delayed scale");
  m.def("layernorm_q8_slots", &ops::layernorm_q8_slots);
  m.def("layernorm_bwd_colsum", &ops::layernorm_bwd_colsum,
        "layernorm backward that also returns per-block column sums of dx (a bias gradient's partials)");
  m.def("qkv_split", &ops::qkv_split);
  m.def("qkv_merge", &ops::qkv_merge);
  m.def("heads_to_rows", &ops::heads_to_rows);
  m.def("rows_to_heads", &ops::rows_to_heads);
  m.def("softmax_fwd", &ops::softmax_fwd);
  m.def("attn_bwd_ds", &ops::attn_bwd_ds, "fused dP = dO V^T + softmax backward -> dS (head dim 64, Tp <= 256)");
  m.def("attn_fwd_rows", &ops::attn_fwd_rows,
        "fused attention forward on the qkv projection rows [B*T, 3*H*64]: returns [P (or, recompute=True, the "
        "per-query log-sum-exp), out rows [B*T, H*64]]",
        py::arg("qkv"), py::arg("B"), py::arg("T"), py::arg("H"), py::arg("scale"), py::arg("recompute") = false);
  m.def("attn_bwd_rows", &ops::attn_bwd_rows, "fused attention backward from output-grad rows -> dqkv rows",
        py::arg("dout"), py::arg("qkv"), py::arg("p"), py::arg("B"), py::arg("T"), py::arg("H"), py::arg("scale"),
        py::arg("colsum_part") = py::none());
  m.def("rowsum_f32", &ops::rowsum_f32, "out[c] = sum_r part[r][c] (fp32, fixed order)");
  m.def("attn_bwd", &ops::attn_bwd,
        "fused attention backward -> dqkv rows [B*T, 3*H*Dh] (query-side dQ kernel + key-side dK/dV kernel)");
  m.def("attn_fwd", &ops::attn_fwd, "fused attention forward (head dim 64, Tp <= 256): returns [P, O]");
  m.def("softmax_bwd", &ops::softmax_bwd);
  m.def("gelu_bwd", &ops::gelu_bwd);
  m.def("assemble_tokens", &ops::assemble_tokens);
  m.def("assemble_tokens_bwd", &ops::assemble_tokens_bwd);
  m.def("cls_rows", &ops::cls_rows);
  m.def("patchify", &ops::patchify);
  m.def("fp8_quantize", &ops::fp8_quantize);
  m.def("fp8_quantize_both", &ops::fp8_quantize_both);
  m.def("fp8_quantize_both_delayed", &ops::fp8_quantize_both_delayed, py::arg("x"), py::arg("hist"), py::arg("init"),
        py::arg("colsum") = py::none(), py::arg("gelu_pre") = py::none(), py::arg("roll") = true);
  m.def("fp8_roll_many", &ops::fp8_roll_many, "delayed-scaling roll of many fp8 sites in one launch");
  m.def("gemm_fp8_q8_slots", &ops::gemm_fp8_q8_slots);
  m.def("fp8_roll", &ops::fp8_roll, "delayed-scaling roll of one fp8 site");
  m.def("fp8_quantize_weights", &ops::fp8_quantize_weights,
        "delayed-scaling e4m3 copies (q, q^T, scale) of many fp32 weights in one launch");
  m.def("gemm_fp8_quant_out", &ops::gemm_fp8_quant_out, py::arg("a"), py::arg("b"), py::arg("scale_a"),
        py::arg("scale_b"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("bias") = py::none(), py::arg("act") = 0,
        py::arg("preact") = py::none(), py::arg("hist"), py::arg("colsum") = py::none());
  m.def("colsum_f32", &ops::colsum_f32, "out[c] = sum_r x[r][c] (bf16 in, fp32 out, deterministic)");
  m.def("fp8_delayed_slots", &ops::fp8_delayed_slots);
  m.def("gemm_fp8", &ops::gemm_fp8, py::arg("a"), py::arg("b"), py::arg("scale_a"), py::arg("scale_b"), py::arg("M"),
        py::arg("N"), py::arg("K"), py::arg("out_bf16") = true, py::arg("bias") = py::none(), py::arg("act") = 0,
        py::arg("residual") = py::none(), py::arg("preact") = py::none());
  m.def("gemm_fp8_splitk_f32", &ops::gemm_fp8_splitk_f32);
  m.def("set_bf16_tile_mode", &ops::set_bf16_tile_mode, "0 auto, 128 / 256: force the bf16 GEMM tile kernel");
  m.def("set_gemm256_phased", &kern::set_gemm256_phased, "K-contiguous 256x256 GEMM: 1 phased pipeline, 0 older kernel");
  m.def("set_gemm_two_wg", &kern::set_gemm_two_wg, "bf16 K-contiguous GEMMs on the 2-workgroup 256x128 kernel: 0 never (default), 1 always, 2 N <= 1024; group_m > 0 sets its tile-order group",
        py::arg("mode"), py::arg("group_m") = 0);
  m.def("set_gemm_store_cache", &kern::set_gemm_store_cache, "256x256 GEMM 16-B output stores: 0 plain, 1 nt, 2 sc1");
  m.def("set_gemm256_persist", &kern::set_gemm256_persist, "K-contiguous 256x256 GEMM: 1 persistent phased kernel, 0 one workgroup per tile");
  m.def("set_gemm_wide_store", &kern::set_gemm_wide_store, "256x256 GEMM epilogue: 1 16-B bf16 stores, 0 8-B stores");
  m.def("set_fp8_tile_mode", &ops::set_fp8_tile_mode,
        "fp8 GEMM kernel choice: 0 auto, 128 the generic 128x128 core, 256 the 256x256 DMA-pipelined kernel");
  m.def("f32_conv_fwd", &ops::f32_conv_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("pad"),
        py::arg("mean") = 0.0, py::arg("std") = 1.0);
  m.def("f32_conv_pool_fwd", &ops::f32_conv_pool_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("pad"),
        py::arg("mean") = 0.0, py::arg("std") = 1.0, py::arg("stride") = 2,
        "conv + bias + ReLU + 2x2 max-pool (stride 2 or 1) in one launch: (pooled activation, 1-byte argmax code)");
  m.def("f32_conv1_pool_fwd", &ops::f32_conv1_pool_fwd, py::arg("x"), py::arg("w1"), py::arg("b1"), py::arg("mean"),
        py::arg("std"), "ConvNet conv1 + ReLU + pool1 at fp32, one wave per image: (a1, code1)");
  m.def("f32_conv1_wgrad", &ops::f32_conv1_wgrad, py::arg("x"), py::arg("da1"), py::arg("code1"), py::arg("mean"),
        py::arg("std"), py::arg("dw1"), py::arg("db1"),
        "ConvNet conv1 weight + bias gradient at fp32 from the pooled gradient (pool backward folded in)");
  m.def("f32_conv_dgrad", &ops::f32_conv_dgrad);
  m.def("f32_conv_wgrad", &ops::f32_conv_wgrad, py::arg("dz"), py::arg("x"), py::arg("pad"), py::arg("mean"),
        py::arg("std"), py::arg("dw"), py::arg("db"));
  m.def("f32_conv_wgrad_slab", &ops::f32_conv_wgrad_slab, py::arg("dz"), py::arg("x"), py::arg("pad"),
        py::arg("mean"), py::arg("std"), py::arg("dw"), py::arg("with_bias"),
        "weight-gradient GEMM with its reduction deferred: (slab, [slices, Kout, Nw, ncol])");
  m.def("f32_conv1_wgrad_slab", &ops::f32_conv1_wgrad_slab);
  m.def("f32_conv_dgrad_pool2s1_bwd", &ops::f32_conv_dgrad_pool2s1_bwd,
        "conv data gradient + the 2x2/s1 pool backward of its input in one pass over the split-K planes");
  m.def("f32_fc_ce_pool3_bwd", &ops::f32_fc_ce_pool3_bwd,
        "fp32 ConvNet head backward: cross entropy + fc1 data gradient + pool3 backward in one launch -> (dl, dz3)");
  m.def("f32_slab_reduce_multi", &ops::f32_slab_reduce_multi,
        "the deferred weight-gradient reductions of several layers in one launch");
  m.def("f32_pool_relu_fwd", &ops::f32_pool_relu_fwd);
  m.def("f32_pool_relu_bwd", &ops::f32_pool_relu_bwd);
  m.def("cn_pack_weights", &ops::cn_pack_weights, py::arg("w1"), py::arg("w2"), py::arg("w3"), py::arg("wfc"),
        py::arg("out") = py::none());
  m.def("cn_conv1_fwd", &ops::cn_conv1_fwd);
  m.def("cn_conv1_fwd_pack", &ops::cn_conv1_fwd_pack);
  m.def("cn_forward_buffers", &ops::cn_forward_buffers);
  m.def("cn_forward_fused", &ops::cn_forward_fused, py::arg("x"), py::arg("w1"), py::arg("b1"), py::arg("w2"),
        py::arg("b2"), py::arg("w3"), py::arg("b3"), py::arg("wfc"), py::arg("bfc"), py::arg("mean"), py::arg("std"),
        py::arg("in_scale"), py::arg("a1"), py::arg("idx1"), py::arg("a2"), py::arg("idx2"), py::arg("packed"),
        py::arg("do_pack") = true);
  m.def("cn_conv2_fwd", &ops::cn_conv2_fwd);
  m.def("cn_conv3_fc_fwd", &ops::cn_conv3_fc_fwd);
  m.def("cn_conv3_fc_bwd", &ops::cn_conv3_fc_bwd, py::arg("a2"), py::arg("idx2"), py::arg("a3"), py::arg("idx3"),
        py::arg("wfc"), py::arg("dlogits"), py::arg("packed"), py::arg("need_dz2"), py::arg("dw3"), py::arg("db3"),
        py::arg("dwfc"), py::arg("dbfc"), py::arg("defer_reduce") = false);
  m.def("cn_conv3_fc_ce_bwd", &ops::cn_conv3_fc_ce_bwd);
  m.def("cn_flush_reduce", &ops::cn_flush_reduce);
  m.def("cn_reduce_pending", &ops::cn_reduce_pending);
  m.def("cn_merged_reductions", &ops::cn_merged_reductions);
  m.def("cn_conv2_bwd", &ops::cn_conv2_bwd);
  m.def("cn_conv1_wgrad", &ops::cn_conv1_wgrad);
  m.def("cn_conv12_bwd", &ops::cn_conv12_bwd);
  m.def("synth_u8_images", &ops::synth_u8_images);
}
