"""Known-bytes calibration launch for rocprofv3 FETCH_SIZE/WRITE_SIZE on gfx950: the stateless
lbsim_reservoir_features kernel over N reservoirs reads exactly 2 x 512 B (values, ts; dword per
lane, 256 B per wave instruction — the same access shape as observe_kernel) + 4 B count per
reservoir and writes 20 B.  python tools/pmc_calib.py [N]"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from marllb_amd import _lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 21
v = torch.rand((n, 128), device="cuda:0")
t = torch.randint(0, 1 << 20, (n, 128), device="cuda:0", dtype=torch.int32)
c = torch.full((n,), 1000, device="cuda:0", dtype=torch.int32)
out = torch.empty((n, 5), device="cuda:0")
torch.cuda.synchronize()
for _ in range(3):
    assert _lib.load().lbsim_reservoir_features(v.data_ptr(), t.data_ptr(), c.data_ptr(), n, 0.9,
                                                out.data_ptr(), None) == 0
torch.cuda.synchronize()
print({"reservoirs": n, "read_bytes": n * (2 * 512 + 4), "write_bytes": n * 20})
