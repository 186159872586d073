"""The XOR-network generator (reed-solomon-erasure_amd/csrc/rse_netgen.hpp)
on the CPU: every network it emits, greedy or exact factoring, any budget,
expands back to the bit matrices of the codec's parity coefficients
(core.rs:430-436 rows; the kernels' correctness rests on this), and the exact
factoring never costs more ops.  Built with g++ from tests/native."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "reed-solomon-erasure_amd", "csrc")


def test_networks_expand_to_the_coefficient_matrices(tmp_path):
    exe = tmp_path / "netgen_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", CSRC,
                    os.path.join(HERE, "native", "netgen_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip().endswith("OK")
    # the generator's headline: GF(2^16) 20+8 at the compiled budget
    line = [x for x in out.stdout.splitlines() if x.startswith("field 16 20+8 budget 32")][0]
    assert "exact 3144" in line, line
