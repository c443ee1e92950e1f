"""ResizeWrapper.forward restated in torch-CPU (reference ModelWrapper.py:12-53).  TEST INFRASTRUCTURE ONLY.

Parity unpinned: the reference forward cannot run (torch.max on a torch.Size at :13, a float interpolate size at
:16-25, the file ends at `result =` on :53), so there is no reference output to pin against.  This restatement follows
the lines one by one with the readings ModelWrapper.py's docstring states (Python max of (H, W); int() of the resized
shorter side; the pad measured on the shorter side, the one :39-48 pads; `result = self.model(input)`).
"""
import math

import torch
import torch.nn.functional as F


def resize_pad_ref(x, larger_side_size=1024, sizes=(256, 512, 1024, 2048)):
    sizes_t = torch.tensor(list(sizes))                                   # :10
    larger = max(int(x.size(2)), int(x.size(3)))                          # :13
    resize_ratio = float(larger_side_size) / larger                       # :14
    smaller = min(int(x.size(2)), int(x.size(3)))                         # :15
    smaller_tgt = smaller * resize_ratio                                  # :16
    if x.size(2) > x.size(3):                                             # :20-23
        tgt = (larger_side_size, int(smaller_tgt))
    else:
        tgt = (int(smaller_tgt), larger_side_size)
    y = F.interpolate(x, size=tgt, mode='bilinear')                       # :25 (align_corners None = False)
    valid = sizes_t[sizes_t > smaller_tgt]                                # :27-28
    cls = int(torch.min(valid))                                           # :29
    portrait = x.size(2) > x.size(3)
    diff = float(cls - (y.size(3) if portrait else y.size(2)))            # :31 (the shorter side; see module doc)
    if portrait:                                                          # :39-43
        pad = (int(math.floor(diff / 2)), int(math.ceil(diff / 2)), 0, 0)
    else:                                                                 # :44-48
        pad = (0, 0, int(math.floor(diff / 2)), int(math.ceil(diff / 2)))
    return F.pad(y, pad=pad)                                              # :50-51


def resize_wrapper_ref(model, x, larger_side_size=1024):
    return model(resize_pad_ref(x, larger_side_size))                     # :53 completed as self.model(input)
