function [t_accepted] = ode23_packets_gpu(hctx, tspan, tmax, f, Cg, nslots)
% ode23_packets_gpu  MATLAB ode23's step-size controller (Bogacki-Shampine
% 3(2), defaults RelTol 1e-3, AbsTol 1e-6, MaxStep 0.1*|tspan|, max-norm)
% over the packets resident on the GPU of context hctx (swrt_mex('packets_set', hctx, ...)), with
% every stage on the device.  Replaces, in qgsw_raytrace.m:143-150 /
% qg2layersw_raytrace.m:189-196,
%   [~, solver_y] = ode23(ray_ode, [0, dt], y0);
% by
%   ode23_packets_gpu(hctx, [0, dt], dt, f, Cg, 2);  [packet_x, packet_k] = swrt_mex('packets_get', hctx);
% with the two grid_U snapshots in slots 0/1 (swrt_mex('qg_snapshot', hctx, ...)).
rtol = max(1e-3, 100*eps); atol = 1e-6; bump = 1e-10;
thr = atol / rtol; pw = 1/3;
t0 = tspan(1); tfinal = tspan(2); tdir = sign(tfinal - t0);
htspan = abs(tfinal - t0); hmax = 0.1 * htspan;
t = t0;
rh = swrt_mex('ode23_f1', hctx, t, tmax, f, Cg, nslots, thr, bump) / (0.8 * rtol^pw);
absh = min(hmax, htspan);
if absh * rh > 1, absh = 1 / rh; end
absh = max(absh, 16*eps(t));
t_accepted = t; done = false;
while ~done
  hmin = 16*eps(t);
  absh = min(hmax, max(hmin, absh));
  h = tdir * absh;
  if 1.1*absh >= abs(tfinal - t), h = tfinal - t; absh = abs(h); done = true; end
  nofailed = true;
  while true
    tnew = t + h;
    if done, tnew = tfinal; end
    err = absh * swrt_mex('ode23_attempt', hctx, t, h, tnew, tmax, f, Cg, nslots, thr, bump);
    h = tnew - t;
    if err > rtol
      if absh <= hmin, error('swrt:ode23', 'step size below hmin at t=%g', t); end
      if nofailed
        nofailed = false; absh = max(hmin, absh * max(0.5, 0.8*(rtol/err)^pw));
      else
        absh = max(hmin, 0.5 * absh);
      end
      h = tdir * absh; done = false;
    else
      break;
    end
  end
  swrt_mex('ode23_accept', hctx);
  t = tnew; t_accepted(end+1) = t; %#ok<AGROW>
  if done, break; end
  if nofailed
    temp = 1.25*(err/rtol)^pw;
    if temp > 0.2, absh = absh / temp; else, absh = 5.0*absh; end
  end
end
end
