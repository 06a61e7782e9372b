"""Debug helper (GPU box): eps of 1024 poses with the library DPK_LIB selects -> .npy"""
import sys

import numpy as np
import torch

sys.path.insert(0, "diffpose-nw_amd")
from diffpose_amd.data import synthetic_batch  # noqa: E402
from diffpose_amd.gcndiff import HipGCNdiff, adj_mx_from_edges  # noqa: E402
from diffpose_amd.weights import synthetic_state_dict  # noqa: E402

m = HipGCNdiff(adj_mx_from_edges(), None, device="cuda:0")
m.load_state_dict(synthetic_state_dict())
x = torch.from_numpy(synthetic_batch(1024, seed=1)[0]).cuda()
t = (torch.arange(1024, dtype=torch.float32) % 50).cuda()
e = m(x, torch.ones(1, 1, 17, dtype=torch.bool, device="cuda:0"), t, 0).cpu().numpy()
np.save(sys.argv[1], e)
