set -o pipefail
python -c "import torch; print('torch first:', torch.cuda.is_available())"
python -c "
import ctypes; ctypes.CDLL('/opt/rocm/lib/libamdhip64.so.7')
import torch; print('rocm first:', torch.cuda.is_available())"
python -c "
import torch, myscaledb_amd as m, numpy as np
m.init(0)
print('after mqvs:', torch.cuda.is_available())
seg = m.VectorScanSegment.from_rows(np.random.rand(1000,16).astype(np.float32), 'L2', 256)
print(seg.search(np.random.rand(2,16).astype(np.float32), 3))
import subprocess; print(open('/proc/%d/maps' % __import__('os').getpid()).read().count('libamdhip64'))
for l in open('/proc/%d/maps' % __import__('os').getpid()):
    if 'libamdhip64' in l: print(l.split()[-1]); break
"
