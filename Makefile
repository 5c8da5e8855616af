# Top-level build.  Everything is compiled for gfx950 only.
#   lib   : dynamic_direct_lidar_odometry_amd/_lib/libddlo_gicp.so (the product: HIP kernels + C-ABI)
#   oracle: oracle/liboracle.so and oracle/_ref/libref_nanoflann.so (TEST-ONLY checker)
#   facade: tests/cpp/facade_replay (C++ NanoGICP facade driver, links the product)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := dynamic_direct_lidar_odometry_amd
CSRC := $(PKG)/csrc
LIBDIR := $(PKG)/_lib
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function
OBJS := $(LIBDIR)/kernels.o $(LIBDIR)/knn_tasks.o $(LIBDIR)/nftree.o $(LIBDIR)/cellgrid.o $(LIBDIR)/tietree.o $(LIBDIR)/capi.o $(LIBDIR)/preprocess.o $(LIBDIR)/odom.o $(LIBDIR)/segment.o

all: lib oracle facade raycast

lib: $(LIBDIR)/libddlo_gicp.so

$(LIBDIR)/kernels.o: $(CSRC)/kernels.hip $(CSRC)/search.hpp $(CSRC)/nn_tasks.hpp $(CSRC)/cov_math.hpp $(CSRC)/gicp_types.hpp $(CSRC)/launch.hpp
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/knn_tasks.o: $(CSRC)/knn_tasks.hip $(CSRC)/search.hpp $(CSRC)/nn_tasks.hpp $(CSRC)/cov_math.hpp $(CSRC)/gicp_types.hpp $(CSRC)/launch.hpp
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/nftree.o: $(CSRC)/nftree.hip $(CSRC)/nftree.hpp $(CSRC)/cov_math.hpp $(CSRC)/gicp_types.hpp $(CSRC)/launch.hpp
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/cellgrid.o: $(CSRC)/cellgrid.hip $(CSRC)/cellgrid.hpp $(CSRC)/search.hpp $(CSRC)/gicp_types.hpp
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/tietree.o: $(CSRC)/tietree.hip $(CSRC)/gicp_types.hpp $(CSRC)/launch.hpp
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/capi.o: $(CSRC)/capi.hip $(CSRC)/nftree.hpp $(CSRC)/runtime.hpp $(CSRC)/cellgrid.hpp $(CSRC)/gicp_types.hpp $(CSRC)/launch.hpp include/ddlo_gicp.h
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/preprocess.o: $(CSRC)/preprocess.hip $(CSRC)/gicp_types.hpp $(CSRC)/launch.hpp
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/odom.o: $(CSRC)/odom.hip $(CSRC)/runtime.hpp $(CSRC)/gicp_types.hpp $(CSRC)/launch.hpp include/ddlo_gicp.h include/ddlo_odom.h
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/segment.o: $(CSRC)/segment.hip $(CSRC)/runtime.hpp $(CSRC)/gicp_types.hpp $(CSRC)/launch.hpp include/ddlo_gicp.h include/ddlo_segment.h
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/libddlo_gicp.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -Wl,--no-undefined -o $@ $(OBJS)

oracle:
	$(MAKE) -C oracle

# test / bench infrastructure: the GPU twin of scene.py's ray caster (cfg 5 frame synthesis)
raycast: tools/raycast/libddlo_raycast.so

tools/raycast/libddlo_raycast.so: tools/raycast/raycast.hip
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<

facade: tests/cpp/facade_replay

tests/cpp/facade_replay: tests/cpp/facade_replay.cpp include/nano_gicp/nano_gicp.hpp include/ddlo_gicp.h $(LIBDIR)/libddlo_gicp.so
	g++ -std=c++17 -O2 -Iinclude -o $@ tests/cpp/facade_replay.cpp -L$(LIBDIR) -lddlo_gicp -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'

clean:
	rm -f $(LIBDIR)/*.o $(LIBDIR)/*.so tests/cpp/facade_replay tools/raycast/libddlo_raycast.so
	$(MAKE) -C oracle clean

.PHONY: all lib oracle facade raycast clean

# developer variant: k_lm_step prints per-phase cycle counts (load with DDLO_GICP_LIB)
lmprof: $(OBJS)
	@mkdir -p $(LIBDIR)/lmprof
	$(HIPCC) $(HIPFLAGS) -DDDLO_LM_PROF -c $(CSRC)/kernels.hip -o $(LIBDIR)/lmprof/kernels.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(LIBDIR)/lmprof/libddlo_gicp.so $(LIBDIR)/lmprof/kernels.o $(filter-out $(LIBDIR)/kernels.o,$(OBJS))

.PHONY: lmprof

# developer variant: the search kernels fill the per-sub-group counters of
# gicp_debug_stats (tools/probe_tasks.py; load with DDLO_GICP_LIB)
statsprof: $(OBJS)
	@mkdir -p $(LIBDIR)/statsprof
	$(HIPCC) $(HIPFLAGS) -DDDLO_SEARCH_STATS -c $(CSRC)/kernels.hip -o $(LIBDIR)/statsprof/kernels.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(LIBDIR)/statsprof/libddlo_gicp.so $(LIBDIR)/statsprof/kernels.o $(filter-out $(LIBDIR)/kernels.o,$(OBJS))

.PHONY: statsprof

# developer variant: k_covariances2 stores per-group stamps (tools/cov_timeline.py; load with DDLO_GICP_LIB)
covprof: $(OBJS)
	@mkdir -p $(LIBDIR)/covprof
	$(HIPCC) $(HIPFLAGS) -DDDLO_COV_PROF -DDDLO_DEV -c $(CSRC)/kernels.hip -o $(LIBDIR)/covprof/kernels.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(LIBDIR)/covprof/libddlo_gicp.so $(LIBDIR)/covprof/kernels.o $(filter-out $(LIBDIR)/kernels.o,$(OBJS))

.PHONY: covprof

# development build: the A/B environment knobs (devknobs.hpp) are read
dev:
	@mkdir -p $(LIBDIR)/dev
	for f in $(notdir $(OBJS:.o=)); do $(HIPCC) $(HIPFLAGS) -DDDLO_DEV -c $(CSRC)/$$f.hip -o $(LIBDIR)/dev/$$f.o || exit 1; done
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(LIBDIR)/dev/libddlo_gicp.so $(addprefix $(LIBDIR)/dev/,$(notdir $(OBJS)))

.PHONY: dev
