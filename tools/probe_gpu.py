import sys, time
sys.path.insert(0, 'deep-multimodal-fusion-of-dce-mri-and-dwi-for-automated-breast-tumor-classification-w.-foundation_amd')
import torch
t0=time.time()
print("cuda", torch.cuda.is_available(), torch.cuda.get_device_name(0), flush=True)
import dmf_native as n
y = torch.empty(1000, device='cuda')
n.call('dmf_iota_f32', n.ptr(y), 1000, 2.0, 1.0, n.stream_ptr())
torch.cuda.synchronize()
ref = torch.arange(1000, device='cuda', dtype=torch.float32)*2+1
print("iota ok", torch.equal(y, ref), time.time()-t0)
import os; print("cpus", os.cpu_count(), "threads", torch.get_num_threads())
