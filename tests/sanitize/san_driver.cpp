// TEST INFRASTRUCTURE: host-only driver built with -fsanitize=address,undefined
// by tests/test_sanitize.py.  It links the CPU oracle (oracle/kfx_oracle.cpp)
// and the dataset front-end (slam-kinectfusion_amd/csrc/kfx_dataset.cpp, the
// PNG/zlib decoder that parses untrusted files) and exercises them on inputs
// the test writes: any sanitizer report aborts with a non-zero exit.
//
//   san_driver pipe <params.bin> <intr.bin> <frames.bin> <n>  oracle pipeline + extract / mesh / render
//   san_driver png <file>...                                  kfx_png_* on each file (errors allowed)
//   san_driver intr <file>...                                 kfx_parse_intr on each file
//   san_driver dataset <dir>                                  kfx_dataset_* over a directory
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/kfx.h"
#include "../../oracle/kfx_oracle.h"

namespace kfx {
static std::string g_err;
void set_error_text(const std::string &msg) { g_err = msg; }  // kfx_api.hip's, for the front-end alone
}  // namespace kfx

static std::vector<char> slurp(const char *path) {
  std::vector<char> b;
  FILE *f = std::fopen(path, "rb");
  if (!f) std::exit(3);
  char buf[1 << 16];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + n);
  std::fclose(f);
  return b;
}

static int run_pipe(char **a) {
  std::vector<char> pb = slurp(a[0]), ib = slurp(a[1]), fb = slurp(a[2]);
  const int n = std::atoi(a[3]);
  if (pb.size() != sizeof(kfx_params) || ib.size() != sizeof(kfx_intrinsics)) return 4;
  kfx_params p;
  kfx_intrinsics in;
  std::memcpy(&p, pb.data(), sizeof p);
  std::memcpy(&in, ib.data(), sizeof in);
  const size_t np = (size_t)in.width * in.height, fbytes = np * 4 + np * 3;
  if (fb.size() != fbytes * (size_t)n) return 5;
  kfo_pipe *pp = kfo_pipe_create(&in, &p);
  for (int k = 0; k < n; ++k) {
    const char *f = fb.data() + fbytes * k;
    std::vector<float> d(np);
    std::memcpy(d.data(), f, np * 4);
    const int st = kfo_pipe_process(pp, reinterpret_cast<const uint8_t *>(f + np * 4), d.data());
    std::printf("frame %d status %d\n", k, st);
  }
  for (int i = 0; i < kfo_pipe_pose_count(pp); ++i) {
    kfx_pose q;
    kfo_pipe_get_pose(pp, i, &q);
    char buf[512];
    kfo_format_pose(&q, buf, sizeof buf);
    std::printf("%s", buf);
  }
  const float vs[3] = {p.volu_range[0] / p.volu_dims[0], p.volu_range[1] / p.volu_dims[1],
                       p.volu_range[2] / p.volu_dims[2]};
  const int64_t cap = 1 << 20;
  std::vector<float> pts(3 * (size_t)cap), tris(9 * (size_t)cap);
  const int Z = p.volu_dims[2];
  const int64_t npts = kfo_extract_points(kfo_pipe_tsdf(pp), kfo_pipe_weight(pp), p.volu_dims, vs, &p.volu_pose,
                                          0, Z, pts.data(), cap);
  const int64_t ntri = kfo_extract_mesh(kfo_pipe_tsdf(pp), kfo_pipe_weight(pp), p.volu_dims, vs, &p.volu_pose,
                                        0, Z, tris.data(), cap);
  std::vector<uint8_t> img(np * 3);
  const float eye[3] = {0.f, 0.f, 0.f};
  kfo_render(kfo_pipe_map(pp, 1, 1, 0), kfo_pipe_map(pp, 1, 2, 0), in.width, in.height, eye, 0, img.data());
  std::printf("points %lld triangles %lld\n", (long long)npts, (long long)ntri);
  kfo_pipe_destroy(pp);
  return 0;
}

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  const std::string mode = argv[1];
  if (mode == "pipe" && argc == 6) return run_pipe(argv + 2);
  if (mode == "png") {
    for (int i = 2; i < argc; ++i) {
      int w = 0, h = 0, c = 0, b = 0;
      const int r = kfx_png_info(argv[i], &w, &h, &c, &b);
      int r1 = -99, r2 = -99;
      if (r == KFX_OK && (size_t)w * h <= (1u << 24)) {
        std::vector<uint8_t> bgr((size_t)w * h * 3);
        std::vector<float> d((size_t)w * h);
        r1 = kfx_png_read_bgr8(argv[i], bgr.data(), w, h);
        r2 = kfx_png_read_depth(argv[i], d.data(), w, h);
      }
      std::printf("%s info %d %dx%d c%d b%d read %d %d\n", argv[i], r, w, h, c, b, r1, r2);
    }
    return 0;
  }
  if (mode == "intr") {
    for (int i = 2; i < argc; ++i) {
      float v[5] = {0, 0, 0, 0, 0};
      std::printf("%s %d %g %g %g %g %g\n", argv[i], kfx_parse_intr(argv[i], v), v[0], v[1], v[2], v[3], v[4]);
    }
    return 0;
  }
  if (mode == "dataset" && argc == 3) {
    kfx_dataset *ds = nullptr;
    int r = kfx_dataset_open(argv[2], &ds);
    std::printf("open %d\n", r);
    if (r) return 0;
    kfx_intrinsics in;
    int n = 0, has = 0;
    r = kfx_dataset_info(ds, &in, &n, &has);
    std::printf("info %d %d frames %dx%d intr %d\n", r, n, in.width, in.height, has);
    std::vector<uint8_t> bgr((size_t)in.width * in.height * 3);
    std::vector<float> d((size_t)in.width * in.height);
    for (int k = 0; k < n; ++k) std::printf("read %d: %d\n", k, kfx_dataset_read(ds, k, bgr.data(), d.data()));
    kfx_dataset_close(ds);
    return 0;
  }
  return 2;
}
