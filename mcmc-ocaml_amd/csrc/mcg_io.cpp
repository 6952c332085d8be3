// mcg_io.cpp -- Read_write text formats (read_write.ml:19-101) for sampler output.
//
// The reference writes one sample per line: the coordinates, the log-likelihood and the
// log-prior, each with Printf "%g" and separated by single spaces (write_sample,
// read_write.ml:19-24); write_nested prefixes a "log_ev log_dev" line and appends the log
// weight to every row (read_write.ml:58-66).  Both are "rows of doubles, %g, space separated",
// which is what mcg_write_rows produces.  GPU runs emit millions of rows, so rows are formatted
// in parallel blocks (one std::string per block) and written in order.
//
// Reading (read / read_nested, read_write.ml:33-56, 72-101) splits each line on blanks and
// parses every field as a float (Scanf " %g "); a line's field count gives the row width.
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mcg.h"

namespace {

// Printf "%g" of OCaml: C's %g for finite values; OCaml prints nan / inf / -inf
inline void put_g(std::string& s, double v) {
  char b[32];
  int n;
  if (std::isnan(v)) n = std::snprintf(b, sizeof b, "nan");
  else n = std::snprintf(b, sizeof b, "%g", v);
  s.append(b, (size_t)n);
}

void format_block(const double* rows, int64_t r0, int64_t r1, int32_t ncols, std::string& out) {
  out.clear();
  out.reserve((size_t)(r1 - r0) * (size_t)ncols * 12);
  for (int64_t r = r0; r < r1; ++r) {
    const double* row = rows + r * ncols;
    for (int32_t c = 0; c < ncols; ++c) {
      if (c) out.push_back(' ');
      put_g(out, row[c]);
    }
    out.push_back('\n');
  }
}

int nthreads_io() {
  unsigned n = std::thread::hardware_concurrency();
  const char* e = std::getenv("OMP_NUM_THREADS");
  if (e && *e) n = (unsigned)std::max(1, std::atoi(e));
  return (int)std::min(16u, std::max(1u, n));
}

bool is_blank(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\f' || c == '\v'; }

// parse one line [p, e) into vals; returns the field count or -1 on a malformed field
int64_t parse_line(const char* p, const char* e, double* vals, int64_t cap) {
  int64_t n = 0;
  std::string tok;
  while (p < e) {
    while (p < e && is_blank(*p)) ++p;
    if (p >= e) break;
    const char* t = p;
    while (p < e && !is_blank(*p)) ++p;
    tok.assign(t, (size_t)(p - t));
    char* end = nullptr;
    errno = 0;
    const double v = std::strtod(tok.c_str(), &end);
    if (end != tok.c_str() + tok.size()) return -1;
    if (vals && n < cap) vals[n] = v;
    ++n;
  }
  return n;
}

bool slurp(const char* path, std::string& buf) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  char tmp[1 << 16];
  size_t k;
  while ((k = std::fread(tmp, 1, sizeof tmp, f)) > 0) buf.append(tmp, k);
  std::fclose(f);
  return true;
}

// lines after `skip`, blank lines ignored (an empty trailing line is End_of_file)
void split_lines(const std::string& buf, int64_t skip, std::vector<std::pair<size_t, size_t>>& lines) {
  size_t p = 0;
  int64_t ln = 0;
  while (p < buf.size()) {
    size_t q = buf.find('\n', p);
    if (q == std::string::npos) q = buf.size();
    if (ln >= skip) {
      bool blank = true;
      for (size_t i = p; i < q && blank; ++i) blank = is_blank(buf[i]);
      if (!blank) lines.emplace_back(p, q);
    }
    ++ln;
    p = q + 1;
  }
}

}  // namespace

extern "C" {

int mcg_write_rows(const char* path, int32_t append, const char* header, int64_t nrows, int32_t ncols,
                   const double* rows) {
  if (!path || nrows < 0 || ncols < 1 || (nrows > 0 && !rows)) return MCG_EINVAL;
  FILE* f = std::fopen(path, append ? "ab" : "wb");
  if (!f) return MCG_EFAIL;
  bool ok = true;
  if (header) ok = std::fputs(header, f) >= 0;
  const int T = nthreads_io();
  const int64_t block = 16384;
  std::vector<std::string> bufs((size_t)T);
  for (int64_t w0 = 0; ok && w0 < nrows; w0 += block * T) {
    std::vector<std::thread> th;
    int used = 0;
    for (int t = 0; t < T; ++t) {
      const int64_t r0 = w0 + t * block, r1 = std::min(nrows, r0 + block);
      if (r0 >= r1) break;
      ++used;
      th.emplace_back(format_block, rows, r0, r1, ncols, std::ref(bufs[(size_t)t]));
    }
    for (auto& x : th) x.join();
    for (int t = 0; t < used && ok; ++t)
      ok = std::fwrite(bufs[(size_t)t].data(), 1, bufs[(size_t)t].size(), f) == bufs[(size_t)t].size();
  }
  if (std::fclose(f) != 0) ok = false;
  return ok ? MCG_OK : MCG_EFAIL;
}

int mcg_read_rows_shape(const char* path, int64_t skip_lines, int64_t* nrows, int32_t* ncols) {
  if (!path || !nrows || !ncols || skip_lines < 0) return MCG_EINVAL;
  std::string buf;
  if (!slurp(path, buf)) return MCG_EFAIL;
  std::vector<std::pair<size_t, size_t>> lines;
  split_lines(buf, skip_lines, lines);
  *nrows = (int64_t)lines.size();
  *ncols = 0;
  for (size_t i = 0; i < lines.size(); ++i) {
    const int64_t n = parse_line(buf.data() + lines[i].first, buf.data() + lines[i].second, nullptr, 0);
    if (n < 0) return MCG_EFAIL;
    if (i == 0) *ncols = (int32_t)n;
    else if (n != *ncols) return MCG_EFAIL;     // ragged rows: not a Read_write file
  }
  return MCG_OK;
}

int mcg_read_rows(const char* path, int64_t skip_lines, int64_t nrows, int32_t ncols, double* rows,
                  double* header, int32_t nheader) {
  if (!path || nrows < 0 || ncols < 0 || (nrows > 0 && !rows)) return MCG_EINVAL;
  std::string buf;
  if (!slurp(path, buf)) return MCG_EFAIL;
  if (header && nheader > 0) {
    const size_t q = std::min(buf.find('\n'), buf.size());
    if (parse_line(buf.data(), buf.data() + q, header, nheader) < nheader) return MCG_EFAIL;
  }
  std::vector<std::pair<size_t, size_t>> lines;
  split_lines(buf, skip_lines, lines);
  if ((int64_t)lines.size() != nrows) return MCG_EFAIL;
  const int T = nthreads_io();
  std::vector<int> bad((size_t)T, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    th.emplace_back([&, t]() {
      for (int64_t r = t; r < nrows; r += T) {
        const auto& L = lines[(size_t)r];
        if (parse_line(buf.data() + L.first, buf.data() + L.second, rows + r * ncols, ncols) != ncols) {
          bad[(size_t)t] = 1;
          return;
        }
      }
    });
  }
  for (auto& x : th) x.join();
  for (int b : bad)
    if (b) return MCG_EFAIL;
  return MCG_OK;
}

}  // extern "C"
