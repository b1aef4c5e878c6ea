bash tools/gpu_idx_prof.sh iprobe4_noins r03h && bash tools/gpu_idx_prof.sh iprobe4_base r03h
