// Python bindings (pybind11) of the native engine: gol_amd._gol.
//
// Python only orchestrates (process-group bootstrap, tensors, tests, bench);
// the generation loop, kernels, halo schedule, I/O and termination logic are
// native.  Long-running calls release the GIL so in-process ranks can run
// on Python threads.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <optional>
#include <thread>
#include <tuple>

#include "gol/backend.hpp"
#include "gol/cpu_ref.hpp"
#include "gol/decomp.hpp"
#include "gol/engine.hpp"
#include "gol/io.hpp"
#include "gol/numa.hpp"
#include "gol/transport.hpp"

namespace py = pybind11;
using namespace gol;

namespace {

// torch.distributed (or anything else) implemented in Python.  Buffers are
// passed as (address, nbytes) pairs in the backend's address space.
class CallbackTransport final : public Transport {
 public:
  using ExchangeFn = std::function<void(py::list, std::uintptr_t)>;
  using ReduceFn = std::function<void(std::uintptr_t, size_t, std::uintptr_t)>;
  using BarrierFn = std::function<void()>;
  CallbackTransport(int rank, int size, ExchangeFn ex, ReduceFn red, BarrierFn bar)
      : rank_(rank), size_(size), ex_(std::move(ex)), red_(std::move(red)), bar_(std::move(bar)) {}
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  const char* name() const override { return "callback"; }
  void exchange(const std::vector<P2POp>& ops, void* stream) override {
    py::gil_scoped_acquire gil;
    py::list l;
    for (const auto& op : ops)
      l.append(py::make_tuple(op.send, op.peer, reinterpret_cast<std::uintptr_t>(op.buf), op.bytes));
    ex_(l, reinterpret_cast<std::uintptr_t>(stream));
  }
  void allreduce_max_u32(uint32_t* buf, size_t n, void* stream) override {
    py::gil_scoped_acquire gil;
    red_(reinterpret_cast<std::uintptr_t>(buf), n, reinterpret_cast<std::uintptr_t>(stream));
  }
  void barrier() override {
    py::gil_scoped_acquire gil;
    bar_();
  }

 private:
  int rank_, size_;
  ExchangeFn ex_;
  ReduceFn red_;
  BarrierFn bar_;
};

py::array_t<uint8_t> to_array(std::vector<uint8_t>&& v, int64_t rows, int64_t cols) {
  auto* heap = new std::vector<uint8_t>(std::move(v));
  py::capsule owner(heap, [](void* p) { delete static_cast<std::vector<uint8_t>*>(p); });
  return py::array_t<uint8_t>({rows, cols}, {cols, int64_t(1)}, heap->data(), owner);
}

const uint8_t* grid_ptr(const py::array_t<uint8_t, py::array::c_style | py::array::forcecast>& a,
                        int64_t rows, int64_t cols) {
  GOL_REQUIRE(a.ndim() == 2 && a.shape(0) == rows && a.shape(1) == cols,
              "expected a " + std::to_string(rows) + "x" + std::to_string(cols) + " uint8 array");
  return a.data();
}

}  // namespace

PYBIND11_MODULE(_gol, m) {
  m.doc() = "gol-mi355x native engine (CDNA4 HIP kernels, RCCL halos, C++ runtime)";
  py::register_exception<Error>(m, "GolError", PyExc_RuntimeError);

  py::enum_<Layout>(m, "Layout").value("U8", Layout::U8).value("Bits", Layout::Bits);

  py::class_<Extent>(m, "Extent")
      .def_readonly("begin", &Extent::begin)
      .def_readonly("end", &Extent::end)
      .def("size", &Extent::size)
      .def("__repr__", [](const Extent& e) {
        return "Extent(" + std::to_string(e.begin) + ", " + std::to_string(e.end) + ")";
      });

  py::class_<Decomposition>(m, "Decomposition")
      .def(py::init<int64_t, int64_t, int, int, int64_t>(), py::arg("W"), py::arg("H"), py::arg("Px"),
           py::arg("Py"), py::arg("col_unit") = 1)
      .def_static("make", &Decomposition::make, py::arg("W"), py::arg("H"), py::arg("nranks"),
                  py::arg("spec") = "auto", py::arg("col_unit") = 1)
      .def_readonly("W", &Decomposition::W)
      .def_readonly("H", &Decomposition::H)
      .def_readonly("Px", &Decomposition::Px)
      .def_readonly("Py", &Decomposition::Py)
      .def("nranks", &Decomposition::nranks)
      .def("rows", &Decomposition::rows)
      .def("cols", &Decomposition::cols)
      .def("px_of", &Decomposition::px_of)
      .def("py_of", &Decomposition::py_of)
      .def("rank_of", &Decomposition::rank_of)
      .def("neighbors", &Decomposition::neighbors)
      .def("describe", &Decomposition::describe);
  m.def("split_range", &split_range);

  py::class_<TileGeom>(m, "TileGeom")
      .def_static("make", &TileGeom::make)
      .def_readonly("H", &TileGeom::H)
      .def_readonly("W", &TileGeom::W)
      .def_readonly("Dv", &TileGeom::Dv)
      .def_readonly("hw", &TileGeom::hw)
      .def_readonly("pitch", &TileGeom::pitch)
      .def("R", &TileGeom::R)
      .def("Wc", &TileGeom::Wc)
      .def("Wp", &TileGeom::Wp)
      .def("bytes", &TileGeom::bytes);

  // Runtime tuning (gol/tuning.hpp).  Python passes a dict: LifeConfig.tune,
  // make_backend(tune=...), bench.py / gol_amd.cli --tune key=value.
  py::class_<Tuning>(m, "Tuning")
      .def(py::init<>())
      .def_static("from_env", &Tuning::from_env)
      .def("set", py::overload_cast<const std::string&, const std::string&>(&Tuning::set),
           py::return_value_policy::reference_internal)
      .def("get", &Tuning::s)
      .def("is_default", &Tuning::is_default)
      .def("source", &Tuning::source)
      .def("values", &Tuning::values)
      .def("changed", &Tuning::changed)
      .def("summary", &Tuning::summary)
      .def("copy", [](const Tuning& t) { return Tuning(t); });
  m.def("tuning_keys", []() {
    py::list out;
    for (const TuningKey& k : tuning_keys()) {
      py::dict d;
      d["key"] = k.key;
      d["env"] = k.env;
      d["default"] = k.dflt;
      d["type"] = std::string(1, k.type);
      d["class"] = k.cls;
      d["doc"] = k.doc;
      out.append(d);
    }
    return out;
  });

  py::class_<Backend, std::shared_ptr<Backend>>(m, "Backend")
      .def("name", &Backend::name)
      .def("tuning", &Backend::tuning, py::return_value_policy::copy)
      .def("is_device", &Backend::is_device)
      .def("device", &Backend::device)
      .def("stream", [](const Backend& b) { return reinterpret_cast<std::uintptr_t>(b.stream()); })
      .def("synchronize", &Backend::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("bind_thread", &Backend::bind_thread);
  m.def("cpu_backend",
        [](int threads, int drift, std::optional<Tuning> tune) {
          return std::shared_ptr<Backend>(make_cpu_backend(threads, drift, tune ? *tune : Tuning::from_env()));
        },
        py::arg("threads") = 0, py::arg("drift") = -1, py::arg("tune") = py::none());
  m.def("hip_backend",
        [](int device, std::optional<Tuning> tune) {
          return std::shared_ptr<Backend>(make_hip_backend(device, tune ? *tune : Tuning::from_env()));
        },
        py::arg("device") = 0, py::arg("tune") = py::none());
  m.def("hip_available", &hip_available);
  m.def("hip_pci_bus_id", &hip_pci_bus_id);
  m.def("hip_release_errors", &hip_release_errors);
  m.def("hip_uuid", &hip_uuid);
  m.def("parse_cpulist", &parse_cpulist);
  m.def("pci_numa_node", &pci_numa_node);
  m.def("pinned_numa_node", &pinned_numa_node);

  py::class_<Transport, std::shared_ptr<Transport>>(m, "Transport")
      .def("rank", &Transport::rank)
      .def("size", &Transport::size)
      .def("name", &Transport::name)
      .def("comm_count", &Transport::comm_count)
      .def("comm_device", &Transport::comm_device)
      .def("barrier", &Transport::barrier, py::call_guard<py::gil_scoped_release>())
      // Raw access for plumbing tests: ops = [(send, peer, address, bytes)],
      // addresses in the transport's address space (device memory for rccl).
      .def("exchange",
           [](Transport& t, const std::vector<std::tuple<bool, int, std::uintptr_t, size_t>>& ops,
              std::uintptr_t stream) {
             std::vector<P2POp> v;
             for (const auto& [send, peer, addr, bytes] : ops)
               v.push_back({send, peer, reinterpret_cast<void*>(addr), bytes});
             py::gil_scoped_release rel;
             t.exchange(v, reinterpret_cast<void*>(stream));
           })
      .def("allreduce_max_u32",
           [](Transport& t, std::uintptr_t addr, size_t n, std::uintptr_t stream) {
             py::gil_scoped_release rel;
             t.allreduce_max_u32(reinterpret_cast<uint32_t*>(addr), n, reinterpret_cast<void*>(stream));
           });
  m.def("self_transport", []() { return std::shared_ptr<Transport>(new SelfTransport()); });
  py::class_<ThreadHub, std::shared_ptr<ThreadHub>>(m, "ThreadHub").def(py::init<int>());
  m.def("thread_transport",
        [](std::shared_ptr<ThreadHub> hub, int rank, std::shared_ptr<Backend> be, std::optional<Tuning> tune) {
          return std::shared_ptr<Transport>(
              new ThreadTransport(std::move(hub), rank, be.get(), tune ? *tune : Tuning::from_env()));
        },
        py::arg("hub"), py::arg("rank"), py::arg("backend"), py::arg("tune") = py::none(), py::keep_alive<0, 3>());
  m.def("callback_transport",
        [](int rank, int size, CallbackTransport::ExchangeFn ex, CallbackTransport::ReduceFn red,
           CallbackTransport::BarrierFn bar) {
          return std::shared_ptr<Transport>(new CallbackTransport(rank, size, ex, red, bar));
        });
  m.def("rccl_unique_id", []() {
    auto v = rccl_unique_id();
    return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
  });
  m.def("rccl_transport",
        [](py::bytes uid, int rank, int nranks, int device, std::optional<Tuning> tune) {
          std::string s = uid;
          std::vector<uint8_t> v(s.begin(), s.end());
          const Tuning t = tune ? *tune : Tuning::from_env();
          std::shared_ptr<Transport> tr;
          {
            py::gil_scoped_release rel;
            tr = make_rccl_transport(v, rank, nranks, device, t);
          }
          return tr;
        },
        py::arg("uid"), py::arg("rank"), py::arg("nranks"), py::arg("device"), py::arg("tune") = py::none());

  py::class_<EngineConfig>(m, "EngineConfig")
      .def(py::init<>())
      .def_readwrite("W", &EngineConfig::W)
      .def_readwrite("H", &EngineConfig::H)
      .def_readwrite("layout", &EngineConfig::layout)
      .def_readwrite("decomp", &EngineConfig::decomp)
      .def_readwrite("gen_limit", &EngineConfig::gen_limit)
      .def_readwrite("check_similarity", &EngineConfig::check_similarity)
      .def_readwrite("sim_freq", &EngineConfig::sim_freq)
      .def_readwrite("start_gen", &EngineConfig::start_gen)
      .def_readwrite("sim_phase", &EngineConfig::sim_phase)
      .def_readwrite("tmax", &EngineConfig::tmax)
      .def_readwrite("epoch", &EngineConfig::epoch)
      .def_readwrite("poll_gens", &EngineConfig::poll_gens)
      .def_readwrite("overlap", &EngineConfig::overlap)
      .def_readwrite("lagged_poll", &EngineConfig::lagged_poll)
      .def_readwrite("timing_barriers", &EngineConfig::timing_barriers)
      .def_readwrite("self_exchange", &EngineConfig::self_exchange)
      .def_readwrite("u8_compute", &EngineConfig::u8_compute)
      .def_readwrite("graphs", &EngineConfig::graphs)
      .def_readwrite("watchdog_s", &EngineConfig::watchdog_s)
      .def_readwrite("tune", &EngineConfig::tune);

  py::class_<RunResult>(m, "RunResult")
      .def_readonly("generations", &RunResult::generations)
      .def_readonly("executed", &RunResult::executed)
      .def_readonly("first_unchanged", &RunResult::first_unchanged)
      .def_readonly("extinct", &RunResult::extinct)
      .def_readonly("stop_reason", &RunResult::stop_reason)
      .def_readonly("loop_ms", &RunResult::loop_ms)
      .def_readonly("exchanges", &RunResult::exchanges)
      .def_readonly("polls", &RunResult::polls)
      .def_readonly("kernel_launches", &RunResult::kernel_launches)
      .def_readonly("overlapped", &RunResult::overlapped)
      .def_readonly("graph_launches", &RunResult::graph_launches)
      .def_readonly("halo_bytes", &RunResult::halo_bytes)
      .def_readonly("linked_launches", &RunResult::linked_launches)
      .def_readonly("phase_timed", &RunResult::phase_timed)
      .def_readonly("compute_ms", &RunResult::compute_ms)
      .def_readonly("halo_ms", &RunResult::halo_ms)
      .def_readonly("fill_ms", &RunResult::fill_ms)
      .def_readonly("allreduce_ms", &RunResult::allreduce_ms);

  py::class_<Engine>(m, "Engine")
      .def(py::init([](const EngineConfig& c, std::shared_ptr<Backend> be, std::shared_ptr<Transport> tr) {
             return new Engine(c, be.get(), tr.get());
           }),
           py::keep_alive<1, 3>(), py::keep_alive<1, 4>())
      .def_property_readonly("config", &Engine::config, py::return_value_policy::copy)
      .def_property_readonly("rank", &Engine::rank)
      .def_property_readonly("rows", &Engine::rows)
      .def_property_readonly("cols", &Engine::cols)
      .def_property_readonly("decomp", &Engine::decomp)
      .def_property_readonly("geom", &Engine::geom)
      .def_property_readonly("compute_geom", &Engine::compute_geom)
      .def_property_readonly("epoch_depth", &Engine::epoch_depth)
      .def_property_readonly("tmax", &Engine::tmax)
      .def("overlap", &Engine::overlap)
      .def("overlap_mode", &Engine::overlap_mode)
      .def_property_readonly("trial_ms_plain", &Engine::trial_ms_plain)
      .def_property_readonly("trial_ms_trigger", &Engine::trial_ms_trigger)
      .def("poll_mode", &Engine::poll_mode)
      .def_property_readonly("poll_trial_ms_joined", &Engine::poll_trial_ms_joined)
      .def_property_readonly("poll_trial_ms_side", &Engine::poll_trial_ms_side)
      .def_property_readonly("poll_trial_ms_side_steady", &Engine::poll_trial_ms_side_steady)
      .def("triggered_sends", &Engine::triggered_sends)
      .def_property("phase_timing", &Engine::phase_timing, &Engine::set_phase_timing)
      .def("graphs", &Engine::graphs)
      .def_property("generation", &Engine::generation, &Engine::set_generation)
      .def_property_readonly("drift", &Engine::drift)
      .def_property_readonly("drifting", &Engine::drifting)
      .def_property_readonly("row_ring", &Engine::row_ring)
      .def_property_readonly("row_ring_fallback", &Engine::row_ring_fallback)
      .def_property_readonly("via_bits", &Engine::via_bits)
      .def("normalize", &Engine::normalize, py::call_guard<py::gil_scoped_release>())
      .def("current_buffer", [](Engine& e) { return reinterpret_cast<std::uintptr_t>(e.current_buffer()); })
      .def("load_cells",
           [](Engine& e, py::array_t<uint8_t, py::array::c_style | py::array::forcecast> a) {
             const uint8_t* p = grid_ptr(a, e.rows().size(), e.cols().size());
             py::gil_scoped_release rel;
             e.load_cells(p, e.cols().size());
           })
      .def("load_global",
           [](Engine& e, py::array_t<uint8_t, py::array::c_style | py::array::forcecast> a) {
             const uint8_t* p = grid_ptr(a, e.decomp().H, e.decomp().W);
             py::gil_scoped_release rel;
             e.load_global(p, e.decomp().W);
           })
      .def("store_cells",
           [](Engine& e, bool ascii) {
             std::vector<uint8_t> v(size_t(e.rows().size() * e.cols().size()));
             {
               py::gil_scoped_release rel;
               e.store_cells(v.data(), e.cols().size(), ascii);
             }
             return to_array(std::move(v), e.rows().size(), e.cols().size());
           },
           py::arg("ascii") = false)
      // Owned rows [r0, r0 + n) only (a band of a grid too large for a host copy).
      .def("store_rows",
           [](Engine& e, int64_t r0, int64_t n, bool ascii) {
             std::vector<uint8_t> v(size_t(std::max<int64_t>(0, n) * e.cols().size()));
             {
               py::gil_scoped_release rel;
               e.store_rows(v.data(), e.cols().size(), r0, n, ascii);
             }
             return to_array(std::move(v), n, e.cols().size());
           },
           py::arg("r0"), py::arg("n"), py::arg("ascii") = false)
      .def("init_random", &Engine::init_random, py::arg("seed"), py::arg("density") = 0.5,
           py::call_guard<py::gil_scoped_release>())
      .def("alive_count", &Engine::alive_count, py::call_guard<py::gil_scoped_release>())
      .def("run", &Engine::run, py::call_guard<py::gil_scoped_release>())
      .def("advance", &Engine::advance, py::call_guard<py::gil_scoped_release>())
      .def("run_until", &Engine::run_until, py::call_guard<py::gil_scoped_release>())
      .def("halo_exchange", &Engine::halo_exchange, py::call_guard<py::gil_scoped_release>())
      .def("step_block", &Engine::step_block, py::call_guard<py::gil_scoped_release>())
      .def("read_text", [](Engine& e, const std::string& path) {
        std::vector<uint8_t> tile;
        {
          py::gil_scoped_release rel;
          read_text_tile(path, e.decomp().W, e.decomp().H, e.rows(), e.cols(), tile);
          e.load_cells(tile.data(), e.cols().size());
        }
      })
      .def("write_text", [](Engine& e, const std::string& path, bool create) {
        std::vector<uint8_t> tile(size_t(e.rows().size() * e.cols().size()));
        py::gil_scoped_release rel;
        e.store_cells(tile.data(), e.cols().size(), false);
        if (create) create_text_file(path, e.decomp().W, e.decomp().H);
        write_text_tile(path, e.decomp().W, e.decomp().H, e.rows(), e.cols(), tile.data(), e.cols().size());
      }, py::arg("path"), py::arg("create") = true);

  // ---- I/O ----
  m.def("read_text_tile", [](const std::string& path, int64_t W, int64_t H, int64_t r0, int64_t r1,
                             int64_t c0, int64_t c1) {
    std::vector<uint8_t> out;
    {
      py::gil_scoped_release rel;
      read_text_tile(path, W, H, {r0, r1}, {c0, c1}, out);
    }
    return to_array(std::move(out), r1 - r0, c1 - c0);
  });
  m.def("read_text_grid", [](const std::string& path, int64_t W, int64_t H) {
    std::vector<uint8_t> out;
    {
      py::gil_scoped_release rel;
      read_text_grid(path, W, H, out);
    }
    return to_array(std::move(out), H, W);
  });
  m.def("create_text_file", &create_text_file, py::call_guard<py::gil_scoped_release>());
  m.def("write_text_tile",
        [](const std::string& path, int64_t W, int64_t H, int64_t r0, int64_t c0,
           py::array_t<uint8_t, py::array::c_style | py::array::forcecast> a) {
          GOL_REQUIRE(a.ndim() == 2, "expected a 2-D array");
          int64_t nr = a.shape(0), nc = a.shape(1);
          const uint8_t* p = a.data();
          py::gil_scoped_release rel;
          write_text_tile(path, W, H, {r0, r0 + nr}, {c0, c0 + nc}, p, nc);
        });
  m.def("write_text_grid", [](const std::string& path, py::array_t<uint8_t, py::array::c_style | py::array::forcecast> a) {
    GOL_REQUIRE(a.ndim() == 2, "expected a 2-D array");
    int64_t H = a.shape(0), W = a.shape(1);
    const uint8_t* p = a.data();
    py::gil_scoped_release rel;
    write_text_grid(path, W, H, p);
  });
  m.def("generate_text_file", &generate_text_file, py::arg("path"), py::arg("W"), py::arg("H"),
        py::arg("seed") = 1, py::arg("density") = 0.5, py::call_guard<py::gil_scoped_release>());
  m.def("random_grid", [](int64_t W, int64_t H, uint64_t seed, double density) {
    std::vector<uint8_t> v(size_t(W * H));
    uint32_t th = density_thresh(density);
    for (int64_t r = 0; r < H; ++r)
      for (int64_t x = 0; x < W; ++x) v[size_t(r * W + x)] = uint8_t(rng_cell(seed, r, x, th));
    return to_array(std::move(v), H, W);
  }, py::arg("W"), py::arg("H"), py::arg("seed") = 1, py::arg("density") = 0.5);

  // ---- serial reference (src/game.c semantics) ----
  m.def("cpu_reference_run",
        [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> a, int64_t gen_limit,
           bool check_similarity, int sim_freq, int threads) {
          GOL_REQUIRE(a.ndim() == 2, "expected a 2-D array");
          int64_t H = a.shape(0), W = a.shape(1);
          std::vector<uint8_t> g(a.data(), a.data() + W * H);
          RefResult r;
          {
            py::gil_scoped_release rel;
            r = cpu_reference_run(g, W, H, gen_limit, check_similarity, sim_freq, threads);
          }
          return py::make_tuple(r.generations, r.loop_ms, to_array(std::move(g), H, W));
        },
        py::arg("grid"), py::arg("gen_limit") = 1000, py::arg("check_similarity") = true,
        py::arg("sim_freq") = 3, py::arg("threads") = 1);

  // ---- bitop3 / rule emulation (for kernel-level tests) ----
  m.def("rule_words", [](uint32_t a0, uint32_t a1, uint32_t a2, uint32_t b0, uint32_t b1, uint32_t b2,
                         uint32_t c0, uint32_t c1, uint32_t c2) {
    return rule_host(hsum_host(a0, a1, a2), hsum_host(b0, b1, b2), hsum_host(c0, c1, c2), b1);
  });
}
