// hiprtc_probe.cpp -- checks, without a GPU, that hiprtc can build a gfx950
// code object from source using the fixed-width integer types and the gfx950
// builtins the bit-sliced kernels need.
//   hipcc -O1 tools/hiprtc_probe.cpp -lhiprtc -o /tmp/hiprtc_probe && /tmp/hiprtc_probe
#include <hip/hiprtc.h>

#include <chrono>
#include <cstdlib>
#include <fstream>
#include <thread>
#include <sstream>
#include <cstdio>
#include <string>
#include <vector>

static const char* kSrc = R"(
using __hip_internal::uint8_t;
using __hip_internal::uint16_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
using __hip_internal::int32_t;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
template <class T, T... I> struct int_seq {};
template <int N> using make_int_seq = __make_integer_seq<int_seq, int, N>;
template <int... I> __device__ int sum(int_seq<int, I...>) { return (I + ... + 0); }
extern "C" __global__ __launch_bounds__(256, 2) void probe(const uint8_t* in, uint8_t* out, uint64_t n) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i * 16 >= n) return;
  u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in) + i);
  v.x = __builtin_amdgcn_bitop3_b32(v.x, v.y, v.z, 0x96) ^ sum(make_int_seq<5>{});
  v.y = __builtin_amdgcn_perm(v.y, v.x, 0x06040200u);
  uint4 w = make_uint4(v.x, v.y, v.z, v.w);
  if (__ballot(w.x == 0) != 0ull) atomicOr(reinterpret_cast<uint32_t*>(out), 1u);
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(out) + i);
}
)";

static int compile_once(int argc, char** argv, const std::string& file_src);

// With an argument: compile that file instead (e.g. a module dumped by
// RSE_JIT_DUMP=dir) and report the time.  PROBE_THREADS=n: n compiles of it
// at once on n threads of this process (does hiprtc build in parallel?).
int main(int argc, char** argv) {
  std::string file_src;
  if (argc > 1) {
    std::ifstream f(argv[1]);
    std::stringstream ss;
    ss << f.rdbuf();
    file_src = ss.str();
  }
  const char* nt = std::getenv("PROBE_THREADS");
  const int n = nt ? std::atoi(nt) : 1;
  if (n <= 1) return compile_once(argc, argv, file_src);
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  std::vector<int> rc(n);
  for (int i = 0; i < n; ++i)
    th.emplace_back([&, i] { rc[i] = compile_once(argc > 2 ? 2 : argc, argv, file_src); });
  for (auto& t : th) t.join();
  std::printf("%d compiles on %d threads: %.0f ms wall\n", n, n,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  for (int r : rc)
    if (r) return r;
  return 0;
}

static int compile_once(int argc, char** argv, const std::string& file_src) {
  auto t0 = std::chrono::steady_clock::now();
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, argc > 1 ? file_src.c_str() : kSrc, "probe.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) return 2;
  const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
  hiprtcResult r = hiprtcCompileProgram(prog, 3, opts);
  size_t logn = 0;
  hiprtcGetProgramLogSize(prog, &logn);
  if (logn > 1) {
    std::string log(logn, '\0');
    hiprtcGetProgramLog(prog, &log[0]);
    std::printf("log:\n%s\n", log.c_str());
  }
  if (r != HIPRTC_SUCCESS) {
    std::printf("compile failed: %s\n", hiprtcGetErrorString(r));
    return 1;
  }
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  std::vector<char> code(n);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  const double ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  std::printf("ok: %zu-byte code object in %.0f ms\n", n, ms);
  if (argc > 2) {  // write the code object (llvm-objdump -d --mcpu=gfx950 / readelf --notes)
    std::ofstream o(argv[2], std::ios::binary);
    o.write(code.data(), (std::streamsize)n);
  }
  return 0;
}
