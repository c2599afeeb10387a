"""Under `make -C icl-mixed-precision-gmres_amd sanitize-test` (VERDICT r4
#7): the CPU tests run against the ASan/UBSan builds of the host library
(loader, generators, halo partitioner, drivers) and of the oracle. This
checks that those builds are the ones mapped into the process, so a clean
run means the sanitized code ran. Skipped in the ordinary CPU run."""
import ctypes as C
import os

import pytest

pytestmark = pytest.mark.skipif(not os.environ.get("MPG_HOST_LIB"), reason="not the sanitizer run")


def test_sanitized_libraries_are_the_ones_loaded(mpg, oracle):
    mpg.host_lib()
    oracle.lib()
    maps = open("/proc/self/maps").read()
    assert os.environ["MPG_HOST_LIB"] in maps
    assert os.environ["MPG_ORACLE_LIB"] in maps
    assert hasattr(C.CDLL(None), "__asan_init")  # the ASan runtime is in the process
    for lib in (os.environ["MPG_HOST_LIB"], os.environ["MPG_ORACLE_LIB"]):
        syms = os.popen(f"nm -D --undefined-only {lib}").read()
        assert "__asan_report" in syms and "__ubsan_handle" in syms, lib
