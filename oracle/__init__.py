"""ORACLE — test infrastructure only.

CPU restatements of the reference's mixed-precision GMRES path used as the
parity checker (tests/, __graft_entry__.smoke()) and as the reported CPU
baseline (bench.py's cpu_baseline leg). Nothing in the product imports this.

  binding.py   ctypes binding of _build/liboracle.so (C++ restatement over the
               MKL runtime, cpu_gmres.cpp / cpu_blas.cpp)
  gmres_np.py  independent NumPy restatement (small sizes only)
"""
