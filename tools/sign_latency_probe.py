"""50 single-window calls of the HIP sign classifier (for rocprofv3 --kernel-trace --stats)."""
import sys
sys.path.insert(0, "/root/repo/isl-signlanguage-translation_amd")
import numpy as np, torch
from islpose import translate
clf = translate.SignClassifier()
x = torch.from_numpy(np.random.RandomState(0).uniform(0, 600, (1, 20, 156)).astype(np.float32)).cuda()
for _ in range(50):
    clf(x)
torch.cuda.synchronize()
