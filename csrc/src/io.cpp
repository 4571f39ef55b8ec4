#include "gol/io.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstring>

#include "gol/backend.hpp"
#include "gol/parallel.hpp"

namespace gol {
namespace {

struct Fd {
  int fd = -1;
  ~Fd() {
    if (fd >= 0) ::close(fd);
  }
};

[[noreturn]] void sys_fail(const std::string& what, const std::string& path) {
  fail(what + " '" + path + "': " + std::strerror(errno));
}

void pread_all(int fd, void* buf, size_t n, int64_t off, const std::string& path) {
  auto* p = static_cast<uint8_t*>(buf);
  while (n > 0) {
    ssize_t r = ::pread(fd, p, n, off);
    if (r < 0) {
      if (errno == EINTR) continue;
      sys_fail("read", path);
    }
    if (r == 0) fail("input file '" + path + "' is too short for the requested grid");
    p += r;
    n -= size_t(r);
    off += r;
  }
}

void pwrite_all(int fd, const void* buf, size_t n, int64_t off, const std::string& path) {
  auto* p = static_cast<const uint8_t*>(buf);
  while (n > 0) {
    ssize_t r = ::pwrite(fd, p, n, off);
    if (r < 0) {
      if (errno == EINTR) continue;
      sys_fail("write", path);
    }
    p += r;
    n -= size_t(r);
    off += r;
  }
}

// A file may not grow past the process's RLIMIT_FSIZE: the kernel would
// answer ftruncate / pwrite / fallocate with SIGXFSZ, which kills the process
// (a Python caller with it) before any error can be reported.
void check_fsize_limit(int64_t end, const std::string& path) {
  struct rlimit rl;
  if (::getrlimit(RLIMIT_FSIZE, &rl) == 0 && rl.rlim_cur != RLIM_INFINITY && uint64_t(end) > uint64_t(rl.rlim_cur))
    fail("output '" + path + "' needs " + std::to_string(end) + " bytes, beyond the file size limit (RLIMIT_FSIZE " +
         std::to_string(uint64_t(rl.rlim_cur)) + " bytes)");
}

// Backs the byte range [off, off + n) of a file with disk blocks before it is
// written through a shared mapping: a store into a sparse page that the file
// system cannot back (disk or quota full, EIO) raises SIGBUS instead of an
// error.  Returns false when the file system cannot reserve ranges (the
// caller then writes with pwrite, which reports such errors); a reservation
// the file system refuses for lack of space fails here, with its reason.
bool reserve_range(int fd, int64_t off, int64_t n, const std::string& path) {
  if (n <= 0) return true;
  check_fsize_limit(off + n, path);
  // fallocate(2), not posix_fallocate: glibc emulates the latter where the
  // file system lacks the call by writing a zero byte per block, which would
  // race with the other ranks writing their rows of the same file.
  int r;
  do r = ::fallocate(fd, 0, off, n);
  while (r != 0 && errno == EINTR);
  if (r == 0) return true;
  if (errno == EOPNOTSUPP || errno == EINVAL || errno == ENOSYS) return false;
  sys_fail("cannot reserve space for output", path);
}

// A read-only or writable shared mapping of a file range, page-aligned
// (null when the file system refuses to map it: the pread/pwrite paths then
// serve).  Text I/O goes through mappings because buffered pwrite to one file
// serialises on the inode lock, so parallel writers do not scale, and a
// mapping saves the copy into a bounce buffer on the read side.
struct Map {
  uint8_t* base = nullptr;  // file byte `off` is base[off - start]
  int64_t start = 0;
  size_t len = 0;
  Map(int fd, int64_t off, int64_t n, bool write) {
    if (n <= 0) return;
    const int64_t page = ::sysconf(_SC_PAGESIZE);
    start = off / page * page;
    len = size_t(off + n - start);
    void* p = ::mmap(nullptr, len, write ? PROT_READ | PROT_WRITE : PROT_READ, MAP_SHARED, fd, start);
    if (p == MAP_FAILED) {
      len = 0;
      return;
    }
    base = static_cast<uint8_t*>(p);
  }
  ~Map() {
    if (base) ::munmap(base, len);
  }
  uint8_t* at(int64_t off) const { return base + (off - start); }
};

// One row of cells from text: '1' alive, any other byte dead.
inline void cells_from_text(uint8_t* dst, const uint8_t* src, int64_t n) {
  for (int64_t x = 0; x < n; ++x) dst[x] = uint8_t(src[x] == '1');
}
// One row of text from cells given as 0/1 or ASCII '0'/'1'.
inline void text_from_cells(uint8_t* dst, const uint8_t* src, int64_t n) {
  for (int64_t x = 0; x < n; ++x) dst[x] = uint8_t('0' + ((src[x] == 1) | (src[x] == '1')));
}

}  // namespace

void read_text_tile_into(const std::string& path, int64_t W, int64_t H, Extent rows, Extent cols, uint8_t* dst,
                         int64_t ld) {
  GOL_REQUIRE(W > 0 && H > 0, "grid dimensions must be positive");
  GOL_REQUIRE(rows.begin >= 0 && rows.end <= H && cols.begin >= 0 && cols.end <= W, "tile out of range");
  Fd f;
  f.fd = ::open(path.c_str(), O_RDONLY);
  if (f.fd < 0) sys_fail("cannot open input", path);
  struct stat st;
  if (::fstat(f.fd, &st) != 0) sys_fail("cannot stat input", path);
  const int64_t size = st.st_size;
  const int64_t nr = rows.size(), nc = cols.size();
  const int64_t exact = H * (W + 1);

  if (size == exact || size == exact - 1) {
    // Exact layout: every rank reads its rows' subarray at the MPI-IO view's
    // offsets, row * (W + 1) + col (src/game_mpi_async.c:180-199), through a
    // mapping of the whole file, rows in parallel.  Whether the file HAS that
    // layout is a property of the whole file, so every rank checks the same
    // bytes - the line break of every row, whatever its own column range - and
    // all ranks of a decomposed run take the same path (a rank-local check let
    // the last-column ranks fall back to the fgetc parse while the others read
    // fixed offsets, and the tiles disagreed).
    const int64_t nl_rows = size == exact ? H : H - 1;  // the last '\n' may be missing
    Map m(f.fd, 0, size, false);
    std::atomic<bool> bad{false};
    global_pool().parallel_for(nl_rows, [&](int64_t b, int64_t e) {
      for (int64_t r = b; r < e && !bad.load(std::memory_order_relaxed); ++r) {
        uint8_t ch = 0;
        if (m.base)
          ch = *m.at(r * (W + 1) + W);
        else
          pread_all(f.fd, &ch, 1, r * (W + 1) + W, path);
        if (ch != '\n') bad = true;
      }
    }, 4096);
    if (!bad.load()) {
      // Every row is W cell bytes + '\n': read fixed offsets like the
      // reference's MPI-IO builds, '1' alive and any other byte dead.  (A
      // stray line break among a row's cells would leave the serial fgetc
      // loop short of W*H cells, where the reference spins forever - quirk
      // Q8 - so the fixed-offset reading is the defined behaviour for it.)
      global_pool().parallel_for(nr, [&](int64_t b, int64_t e) {
        std::vector<uint8_t> line(m.base ? 0 : size_t(nc));
        for (int64_t i = b; i < e; ++i) {
          const int64_t off = (rows.begin + i) * (W + 1) + cols.begin;
          const uint8_t* src = m.base ? m.at(off) : line.data();
          if (!m.base) pread_all(f.fd, line.data(), size_t(nc), off, path);
          cells_from_text(dst + i * ld, src, nc);
        }
      }, 16);
      return;
    }
  }
  // Sequential fallback with the reference's fgetc semantics (skip '\n'; we
  // also skip '\r' so CRLF files work): cells are the first W*H other bytes.
  std::vector<uint8_t> data(static_cast<size_t>(size));
  if (size > 0) pread_all(f.fd, data.data(), size_t(size), 0, path);
  for (int64_t i = 0; i < nr; ++i) std::memset(dst + i * ld, 0, size_t(nc));
  int64_t k = 0;
  const int64_t need = W * H;
  for (int64_t i = 0; i < size && k < need; ++i) {
    uint8_t ch = data[size_t(i)];
    if (ch == '\n' || ch == '\r') continue;
    int64_t r = k / W, x = k % W;
    if (r >= rows.begin && r < rows.end && x >= cols.begin && x < cols.end)
      dst[(r - rows.begin) * ld + (x - cols.begin)] = uint8_t(ch == '1');
    ++k;
  }
  if (k < need)
    fail("input file '" + path + "' holds " + std::to_string(k) + " cells, need " +
         std::to_string(need) + " (" + std::to_string(W) + "x" + std::to_string(H) + ")");
}

void read_text_tile(const std::string& path, int64_t W, int64_t H, Extent rows, Extent cols,
                    std::vector<uint8_t>& out) {
  GOL_REQUIRE(rows.begin >= 0 && rows.end <= H && cols.begin >= 0 && cols.end <= W, "tile out of range");
  out.resize(size_t(rows.size() * cols.size()));
  read_text_tile_into(path, W, H, rows, cols, out.data(), cols.size());
}

void create_text_file(const std::string& path, int64_t W, int64_t H) {
  Fd f;
  f.fd = ::open(path.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
  if (f.fd < 0) sys_fail("cannot create output", path);
  check_fsize_limit(H * (W + 1), path);
  if (::ftruncate(f.fd, H * (W + 1)) != 0) sys_fail("cannot size output", path);
}

void write_text_tile(const std::string& path, int64_t W, int64_t H, Extent rows, Extent cols,
                     const uint8_t* cells, int64_t ld) {
  Fd f;
  f.fd = ::open(path.c_str(), O_RDWR);
  if (f.fd < 0) sys_fail("cannot open output", path);
  const int64_t nr = rows.size(), nc = cols.size();
  const bool nl = cols.end == W;
  (void)H;
  if (nr <= 0 || nc <= 0) return;
  // The tile's rows through a writable shared mapping of their byte range
  // (the MPI-IO writers' subarray view, src/game_mpi_async.c:382-455), rows
  // converted straight into the page cache in parallel; pwrite per row where
  // the file cannot be mapped or its range not reserved (reserve_range).
  const int64_t first = rows.begin * (W + 1) + cols.begin;
  const int64_t last = (rows.end - 1) * (W + 1) + cols.begin + nc + (nl ? 1 : 0);
  struct stat st;
  const bool sized = ::fstat(f.fd, &st) == 0 && st.st_size >= last;
  check_fsize_limit(last, path);
  Map m(f.fd, first, (sized && reserve_range(f.fd, first, last - first, path)) ? last - first : 0, true);
  global_pool().parallel_for(nr, [&](int64_t b, int64_t e) {
    std::vector<uint8_t> buf(m.base ? 0 : size_t(nc + 1));
    for (int64_t i = b; i < e; ++i) {
      const int64_t off = (rows.begin + i) * (W + 1) + cols.begin;
      uint8_t* d = m.base ? m.at(off) : buf.data();
      text_from_cells(d, cells + i * ld, nc);
      if (nl) d[nc] = '\n';
      if (!m.base) pwrite_all(f.fd, buf.data(), size_t(nc + (nl ? 1 : 0)), off, path);
    }
  }, 16);
}

void generate_text_file(const std::string& path, int64_t W, int64_t H, uint64_t seed,
                        double density) {
  create_text_file(path, W, H);
  Fd f;
  f.fd = ::open(path.c_str(), O_RDWR);
  if (f.fd < 0) sys_fail("cannot open output", path);
  const uint32_t th = density_thresh(density);
  Map m(f.fd, 0, reserve_range(f.fd, 0, H * (W + 1), path) ? H * (W + 1) : 0, true);
  global_pool().parallel_for(H, [&](int64_t b, int64_t e) {
    std::vector<uint8_t> buf(m.base ? 0 : size_t(W + 1));
    for (int64_t r = b; r < e; ++r) {
      uint8_t* d = m.base ? m.at(r * (W + 1)) : buf.data();
      for (int64_t x = 0; x < W; ++x) d[x] = uint8_t('0' + rng_cell(seed, r, x, th));
      d[W] = '\n';
      if (!m.base) pwrite_all(f.fd, buf.data(), buf.size(), r * (W + 1), path);
    }
  }, 16);
}

}  // namespace gol
