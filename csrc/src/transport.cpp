#include "gol/transport.hpp"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "gol/backend.hpp"
#include "gol/common.hpp"

namespace gol {

void SelfTransport::exchange(const std::vector<P2POp>& ops, void*) {
  GOL_REQUIRE(ops.empty(), "SelfTransport cannot exchange with other ranks");
}

ThreadHub::ThreadHub(int nranks) : red(), n_(nranks) { GOL_REQUIRE(nranks > 0, "hub size"); }

ThreadTransport::ThreadTransport(std::shared_ptr<ThreadHub> hub, int rank, Backend* backend, const Tuning& tune)
    : hub_(std::move(hub)), rank_(rank), backend_(backend) {
  delay_us_ = std::max(0, tune.i("fault_delay_us"));
  side_ = tune.on("cpu_side_poll");
  garble_at_ = tune.i("fault_garble");
  rng_ = 0x9E3779B97F4A7C15ull * uint64_t(rank + 1);
}

void ThreadTransport::fault_delay() {
  if (delay_us_ <= 0) return;
  rng_ ^= rng_ << 13;
  rng_ ^= rng_ >> 7;
  rng_ ^= rng_ << 17;
  std::this_thread::sleep_for(std::chrono::microseconds(rng_ % uint64_t(delay_us_ + 1)));
}

// Rendezvous exchange: sends publish the sender's buffer, the receiver copies
// straight out of it (device-to-device for HIP backends on one device) and
// marks it consumed; the sender returns once all its messages are consumed.
void ThreadTransport::exchange(const std::vector<P2POp>& ops, void* stream) {
  // Sender data must be complete before publishing: it may come from the
  // compute stream or from the stream the engine enqueued this exchange on.
  backend_->synchronize();
  if (stream) backend_->synchronize_stream(stream);
  fault_delay();
  std::vector<std::shared_ptr<ThreadHub::Msg>> sent;
  {
    std::lock_guard<std::mutex> lk(hub_->mu);
    for (const auto& op : ops) {
      if (!op.send) continue;
      auto m = std::make_shared<ThreadHub::Msg>();
      m->buf = op.buf;
      m->bytes = op.bytes;
      m->device = backend_->is_device() ? backend_->device() : -1;
      hub_->queues[{rank_, op.peer}].push_back(m);
      sent.push_back(m);
    }
  }
  hub_->cv.notify_all();
  for (const auto& op : ops) {
    if (op.send) continue;
    std::shared_ptr<ThreadHub::Msg> m;
    {
      std::unique_lock<std::mutex> lk(hub_->mu);
      auto& q = hub_->queues[{op.peer, rank_}];
      hub_->cv.wait(lk, [&] { return !q.empty(); });
      m = q.front();
      q.pop_front();
    }
    GOL_REQUIRE(m->bytes == op.bytes, "thread transport: message size mismatch (" +
                                          std::to_string(m->bytes) + " vs " +
                                          std::to_string(op.bytes) + ")");
    fault_delay();
    // Ranks on different GPUs of one process: the receiver's device copies
    // straight out of the sender's buffer over xGMI, which needs peer access
    // (enable_peer throws where the hardware has none).
    const int mine = backend_->is_device() ? backend_->device() : -1;
    if (m->device >= 0 && mine >= 0 && m->device != mine &&
        std::find(peers_enabled_.begin(), peers_enabled_.end(), m->device) == peers_enabled_.end()) {
      backend_->enable_peer(m->device);
      peers_enabled_.push_back(m->device);
    }
    backend_->copy_2d_async(op.buf, int64_t(op.bytes), m->buf, int64_t(op.bytes), int64_t(op.bytes), 1);
    backend_->synchronize();
    if (garble_at_ > 0 && ++received_ == garble_at_ && op.bytes > 0) {
      // flip the low bit of every 8th byte: cells (u8 layout) or bit-cells
      std::vector<uint8_t> h(op.bytes);
      backend_->copy_d2h(h.data(), op.buf, op.bytes);
      for (size_t i = 0; i < h.size(); i += 8) h[i] ^= 0x01;
      backend_->copy_h2d(op.buf, h.data(), op.bytes);
    }
    {
      std::lock_guard<std::mutex> lk(hub_->mu);
      m->consumed = true;
    }
    hub_->cv.notify_all();
  }
  std::unique_lock<std::mutex> lk(hub_->mu);
  hub_->cv.wait(lk, [&] {
    return std::all_of(sent.begin(), sent.end(), [](const auto& m) { return m->consumed; });
  });
}

void ThreadTransport::allreduce_max_u32(uint32_t* buf, size_t n, void* stream) {
  if (stream) backend_->synchronize_stream(stream);  // flags written on that stream
  std::vector<uint32_t> local(n);
  backend_->copy_d2h(local.data(), buf, n * sizeof(uint32_t));
  std::unique_lock<std::mutex> lk(hub_->mu);
  uint64_t gen = hub_->generation;
  if (hub_->arrived == 0) hub_->red.assign(n, 0u);
  GOL_REQUIRE(hub_->red.size() == n, "thread allreduce: size mismatch");
  for (size_t i = 0; i < n; ++i) hub_->red[i] = std::max(hub_->red[i], local[i]);
  if (++hub_->arrived == hub_->size()) {
    hub_->arrived = 0;
    ++hub_->generation;
    hub_->cv.notify_all();
  } else {
    hub_->cv.wait(lk, [&] { return hub_->generation != gen; });
  }
  local = hub_->red;
  lk.unlock();
  // Everybody must have read `red` before the next reduction resets it.
  barrier();
  backend_->copy_h2d(buf, local.data(), n * sizeof(uint32_t));
}

void ThreadTransport::barrier() {
  std::unique_lock<std::mutex> lk(hub_->mu);
  uint64_t gen = hub_->generation;
  if (++hub_->arrived == hub_->size()) {
    hub_->arrived = 0;
    ++hub_->generation;
    hub_->cv.notify_all();
  } else {
    hub_->cv.wait(lk, [&] { return hub_->generation != gen; });
  }
}

}  // namespace gol
