import sys, os, numpy as np
sys.path.insert(0,'ldpc-sims_amd'); sys.path.insert(0,'tests'); sys.path.insert(0,'oracle')
import torch, oracle, ldpc_amd
from ldpc_amd.codes import get_code, Graph
from test_gpu_config2 import _qam16_llrs
from softparity import decoded_rows
H,_=get_code('wifi1944_56')
dec=ldpc_amd.get_decoder(H)
for ebn0 in (6.0, 6.5):
    cw,x=_qam16_llrs(H,256,ebn0,seed=40+int(ebn0*10))
    r=dec.decode(x,50,algo='tanh',clamp=20.0,soft='z')
    llr=x.cpu().numpy()
    ds=oracle.sp_f32(H,llr,50,20.0,stable=True)
    es=oracle.sp_f32(H,llr,50,20.0,stable=True,early_stop=True)
    f64=oracle.sp_f64(H,llr.astype(np.float64),50,20.0,ceiling='f32')
    conv=decoded_rows(np.asarray(H),f64['z'])
    g=r['soft'].cpu().numpy().astype(np.float64)
    sc=np.maximum(1,np.abs(f64['z']))
    eg=np.abs(g-f64['z'])/sc; eo=np.abs(ds['z']-f64['z'])/sc; ego=np.abs(g-ds['z'])/np.maximum(1,np.abs(ds['z']))
    print(ebn0,'decoded',conv.sum(),'gpu-f64 %.2e oracle-f64 %.2e gpu-oracle %.2e'%(eg[conv].max(),eo[conv].max(),ego[conv].max()))
    i,j=np.unravel_index(np.argmax(np.where(conv[:,None],ego,0)),ego.shape)
    print('  worst cw',i,'var',j,'z64',f64['z'][i,j],'gpu',g[i,j],'ds',ds['z'][i,j],'conv iter',es['iters_used'][i], 'llr min/max', llr.min(), llr.max(), 'zeros', int((llr==0).sum()))
    print('  per-cw worst gpu-f64 for decoded rows sorted:', np.sort(eg[conv].max(axis=1))[-5:], 'iters of those', es['iters_used'][conv][np.argsort(eg[conv].max(axis=1))[-5:]])
