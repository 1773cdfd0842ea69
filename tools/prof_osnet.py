"""One OSNet configuration's forward passes, for rocprofv3 --kernel-trace --stats."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from yolo_tracking_amd.appearance.osnet import OSNetReID  # noqa: E402

half = "--half" in sys.argv
hip = "--torch" not in sys.argv
net = OSNetReID("osnet_x0_25", None, device="cuda:0", half=half, hip=hip)
x = torch.randn(1024, 3, 256, 128, device="cuda:0", dtype=torch.float16 if half else torch.float32)
for _ in range(6):
    net(x)
torch.cuda.synchronize()
