grep NSpid /proc/self/status
ls /sys/class/kfd/kfd/proc/
for d in /sys/class/kfd/kfd/proc/*; do echo $d; ls $d; cat $d/vram_* 2>/dev/null; done
timeout -k 5 60 python -c "
import torch,os,glob,time
x=torch.ones(1<<28,device='cuda'); torch.cuda.synchronize()
print('me',os.getpid())
for d in glob.glob('/sys/class/kfd/kfd/proc/*'):
    print(d, [(f, open(f).read().strip()) for f in glob.glob(d+'/vram_*')], os.listdir(d))
"
