"""Tensors across a multiprocessing queue by value.

torch's default sharing strategy passes a CPU tensor's storage as a file descriptor through a listener socket in
the sending process's temp directory; on the GPU boxes the receiving test process could not reach that socket
(FileNotFoundError in multiprocessing.resource_sharer). Workers pack their results into numpy arrays (bf16 as its
int16 bit pattern, so values stay bit-exact) and the parent unpacks them.
"""
import numpy as np
import torch

_TAG = "__tensor__"


def pack(obj):
    if isinstance(obj, torch.Tensor):
        t = obj.detach().cpu().contiguous()
        if t.dtype == torch.bfloat16:
            return (_TAG, t.view(torch.int16).numpy().copy(), "bfloat16")
        return (_TAG, t.numpy().copy(), str(t.dtype).replace("torch.", ""))
    if isinstance(obj, dict):
        return {k: pack(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(pack(v) for v in obj)
    return obj


def unpack(obj):
    if isinstance(obj, tuple) and len(obj) == 3 and obj[0] == _TAG:
        _, a, dtype = obj
        t = torch.from_numpy(np.asarray(a))
        return t.view(torch.bfloat16) if dtype == "bfloat16" else t
    if isinstance(obj, dict):
        return {k: unpack(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(unpack(v) for v in obj)
    return obj
