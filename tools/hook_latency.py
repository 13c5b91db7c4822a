import ctypes as C, os, sys
lib = C.CDLL(os.path.join("/root/repo", "tools", "libbatchload.so"))
lib.bl_hook_latency.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_long, C.POINTER(C.c_double)]
out = (C.c_double * 7)()
print(lib.bl_hook_latency(0, 16, 4, 1200, 4, 2000, out), list(out))
