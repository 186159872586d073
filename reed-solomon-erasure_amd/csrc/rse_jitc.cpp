// rse_jitc.cpp -- compiles one run-time specialised module of rse_jit.cpp in a
// process of its own:
//
//     rse_jitc <source.hip> <output.co> [hiprtc options...]
//
// The library spawns it (rse_jit.cpp build_module) instead of calling hiprtc in
// process, for two reasons: comgr serialises compiles inside one process, so
// separate processes build several modules at once on several cores; and a
// child process can be stopped when the library is unloaded, where an
// in-process hiprtc call would block exit until it returns.  The helper only
// compiles (hiprtc runs on the host CPU and touches no device).
// Exit status 0: the code object was written; 1: compile failed (log on
// stderr); 2: usage or I/O error.
#include <hip/hiprtc.h>

#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <source.hip> <output.co> [options...]\n", argv[0]);
    return 2;
  }
  std::ifstream in(argv[1], std::ios::binary);
  if (!in) {
    std::fprintf(stderr, "rse_jitc: cannot read %s\n", argv[1]);
    return 2;
  }
  std::stringstream ss;
  ss << in.rdbuf();
  const std::string src = ss.str();
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "rse_jit.hip", 0, nullptr, nullptr) !=
      HIPRTC_SUCCESS) {
    std::fprintf(stderr, "rse_jitc: hiprtcCreateProgram failed\n");
    return 1;
  }
  std::vector<const char*> opts(argv + 3, argv + argc);
  const hiprtcResult r = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
  size_t n = 0;
  if (hiprtcGetProgramLogSize(prog, &n) == HIPRTC_SUCCESS && n > 1) {
    std::string log(n, '\0');
    hiprtcGetProgramLog(prog, &log[0]);
    std::fputs(log.c_str(), stderr);
  }
  int status = 1;
  if (r == HIPRTC_SUCCESS && hiprtcGetCodeSize(prog, &n) == HIPRTC_SUCCESS && n > 0) {
    std::string code(n, '\0');
    if (hiprtcGetCode(prog, &code[0]) == HIPRTC_SUCCESS) {
      std::ofstream out(argv[2], std::ios::binary | std::ios::trunc);
      out.write(code.data(), (std::streamsize)code.size());
      status = out.good() ? 0 : 2;
    }
  }
  hiprtcDestroyProgram(&prog);
  return status;
}
