"""ctypes signatures of libhds_host.so (csrc/host/*.cpp)."""
import ctypes

P, I, L, F, D, Z = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_double, ctypes.c_size_t

SIGS = {
    # pinned_ring.cpp
    "hds_host_alloc": (P, [Z, I]),
    "hds_host_free": (I, [P]),
    "hds_ring_create": (P, [Z, I, I]),
    "hds_ring_destroy": (I, [P]),
    "hds_ring_slot_ptr": (P, [P, I]),
    "hds_ring_slot_bytes": (Z, [P]),
    "hds_ring_acquire": (I, [P]),
    "hds_ring_d2h": (I, [P, I, P, Z, Z, P]),
    "hds_ring_h2d": (I, [P, I, P, Z, Z, P]),
    "hds_ring_record": (I, [P, I, P]),
    "hds_ring_wait": (I, [P, I]),
    "hds_ring_stream_wait": (I, [P, I, P]),
    "hds_ring_query": (I, [P, I]),
    "hds_memcpy_async": (I, [P, P, Z, I, P]),
    # ragged_meta.cpp
    "hds_ragged_meta_size": (L, [I, L, I, L]),
    "hds_ragged_meta_build": (L, [P, P, I, P, P, I, I, I, I, P, L, P]),
    # cpu_optim.cpp
    "hds_cpu_adam": (I, [P, P, I, P, P, P, L, F, F, F, F, F, F, F, I, F]),
    "hds_cpu_lion": (I, [P, P, I, P, P, L, F, F, F, F, F]),
    "hds_cpu_adagrad": (I, [P, P, I, P, P, L, F, F, F, F]),
    "hds_cpu_sumsq": (D, [P, I, L, P]),
    "hds_cpu_num_threads": (I, []),
    "hds_cpu_set_num_threads": (I, [I]),
    # shm_comm.cpp
    "hds_shm_open": (P, [ctypes.c_char_p, I, I, L, I]),
    "hds_shm_close": (I, [P, I]),
    "hds_shm_slot_bytes": (L, [P]),
    "hds_shm_allreduce": (I, [P, P, L, I]),
    # aio.cpp
    "hds_aio_create": (P, [L, I, I, I, I]),
    "hds_aio_destroy": (I, [P]),
    "hds_aio_pread": (I, [P, P, L, ctypes.c_char_p, L, I]),
    "hds_aio_pwrite": (I, [P, P, L, ctypes.c_char_p, L, I]),
    "hds_aio_wait": (L, [P]),
    "hds_aio_submit": (L, [P, I, P, L, ctypes.c_char_p, L]),
    "hds_aio_wait_req": (I, [P, L]),
    "hds_aio_engine": (I, [P]),
    "hds_aio_file_size": (L, [ctypes.c_char_p]),
    # rccl_comm.cpp
    "hds_rccl_load": (I, [ctypes.c_char_p]),
    "hds_rccl_error_string": (ctypes.c_char_p, [I]),
    "hds_rccl_unique_id": (I, [ctypes.c_char_p]),
    "hds_rccl_init": (P, [ctypes.c_char_p, I, I, P, ctypes.POINTER(I)]),
    "hds_rccl_destroy": (I, [P]),
    "hds_rccl_stream": (P, [P]),
    "hds_rccl_all_gather": (I, [P, P, P, Z, I, P, ctypes.POINTER(I)]),
    "hds_rccl_reduce_scatter": (I, [P, P, P, Z, I, I, P, ctypes.POINTER(I)]),
    "hds_rccl_all_reduce": (I, [P, P, P, Z, I, I, P, ctypes.POINTER(I)]),
    "hds_rccl_broadcast": (I, [P, P, P, Z, I, I, P, ctypes.POINTER(I)]),
    "hds_rccl_all_to_all": (I, [P, P, P, Z, I, I, P, ctypes.POINTER(I)]),
    "hds_rccl_wait": (I, [P, I, P]),
    "hds_rccl_query": (I, [P, I]),
    "hds_rccl_synchronize": (I, [P]),
}


def bind(lib):
    for name, (res, args) in SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
