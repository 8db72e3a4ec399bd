from .compressed import CompressedBackend, compressed_allreduce, pack_signs, unpack_signs

__all__ = ["CompressedBackend", "compressed_allreduce", "pack_signs", "unpack_signs"]
