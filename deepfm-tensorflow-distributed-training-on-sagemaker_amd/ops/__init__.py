"""Native ops: ctypes bindings to the gfx950 HIP kernel library (csrc/kernels) and the
C++ host I/O library (csrc/io).  See ``_lib.py`` for the loading rules and ``build.py`` for
the in-tree build."""
