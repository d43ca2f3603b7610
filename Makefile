# Build for the MI355X-native object-storage benchmark.
#   make            -> python extension + native tools, all in-tree
# GPU code targets gfx950 only (CDNA4).
PY        ?= python3
HIPCC     ?= /opt/rocm/bin/hipcc
CXX       ?= g++
ARCH      ?= gfx950
PKG       := custom_go_client_benchmark_amd
BUILD     := build
EXT_SUFFIX := $(shell $(PY) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYBIND_INC := $(shell $(PY) -m pybind11 --includes)

CXXSTD   := -std=c++17
OPT      ?= -O3 -g1
HOSTARCH := -march=x86-64-v2 -mtune=generic
WARN     := -Wall -Wextra -Wno-unused-parameter -Wno-missing-field-initializers
CPPFLAGS := -Icsrc -D__HIP_PLATFORM_AMD__ -isystem /opt/rocm/include
CXXFLAGS := $(CXXSTD) $(OPT) $(HOSTARCH) $(WARN) -fPIC -pthread $(EXTRA_CXXFLAGS)
HIPFLAGS := $(CXXSTD) $(OPT) --offload-arch=$(ARCH) -fPIC -pthread -Icsrc -munsafe-fp-atomics $(EXTRA_HIPFLAGS)
LDLIBS   := -lssl -lcrypto -lpthread

CORE_SRCS := csrc/core/crc32c.cc csrc/core/affinity.cc csrc/core/ceiling.cc csrc/core/hugebuf.cc csrc/core/content.cc csrc/core/util.cc csrc/core/json.cc csrc/core/sched_probe.cc \
             csrc/net/socket.cc csrc/net/tcp_chrono.cc csrc/net/buffered.cc \
             csrc/http1/http1.cc csrc/h2/hpack.cc csrc/h2/h2.cc csrc/h2/h2_client.cc csrc/proto/storage_v2.cc \
             csrc/storage/sink.cc csrc/storage/sliced.cc csrc/storage/auth.cc csrc/storage/client.cc csrc/storage/http_client.cc \
             csrc/storage/grpc_client.cc \
             csrc/server/store.cc csrc/server/media.cc csrc/server/fakegcs.cc csrc/server/server_http1.cc csrc/server/server_grpc.cc \
             csrc/gpu/crc_host.cc
GPU_SRCS  := csrc/gpu/crc32c_kernels.hip csrc/gpu/engine.hip csrc/gpu/copy_engines.hip
PY_SRCS   := csrc/py/bindings.cc csrc/bench/runner.cc

CORE_OBJS := $(patsubst csrc/%.cc,$(BUILD)/%.o,$(CORE_SRCS))
GPU_OBJS  := $(patsubst csrc/%.hip,$(BUILD)/%.o,$(GPU_SRCS))
PY_OBJS   := $(patsubst csrc/%.cc,$(BUILD)/%.o,$(PY_SRCS))

EXT := $(PKG)/_native$(EXT_SUFFIX)
TOOLS := fakegcs read_operation ssd_test write_operations list_operation open_file small_poc loopback_ceiling
TOOL_BINS := $(addprefix $(PKG)/bin/,$(TOOLS))

.PHONY: all clean ext tools asan tsan stress
all: ext tools
ext: $(EXT)
tools: $(TOOL_BINS)

$(BUILD)/%.o: csrc/%.cc
	@mkdir -p $(dir $@)
	$(CXX) $(CPPFLAGS) $(CXXFLAGS) $(PYBIND_INC) -MMD -MP -c $< -o $@

$(BUILD)/%.o: csrc/%.hip
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -MMD -MP -c $< -o $@

$(BUILD)/libgcsbcore.a: $(CORE_OBJS)
	@rm -f $@
	ar rcs $@ $^

$(EXT): $(PY_OBJS) $(GPU_OBJS) $(BUILD)/libgcsbcore.a
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(PY_OBJS) $(GPU_OBJS) $(BUILD)/libgcsbcore.a \
	  -L/opt/rocm/lib -lamdhip64 -lhsa-runtime64 -lrocprofiler-sdk-roctx $(LDLIBS) -Wl,-rpath,/opt/rocm/lib

$(PKG)/bin/%: csrc/tools/%.cc $(BUILD)/libgcsbcore.a
	@mkdir -p $(PKG)/bin $(BUILD)/tools
	$(CXX) $(CPPFLAGS) $(CXXFLAGS) -MMD -MP -MF $(BUILD)/tools/$*.d -MT $@ -o $@ $< $(BUILD)/libgcsbcore.a $(LDLIBS)

# Host-side sanitizer builds of the C++ core + a concurrency stress driver
# (csrc/tests/stress.cc).  GPU code is not sanitized (no GPU ASan on this pool).
SAN_SRCS := $(CORE_SRCS) csrc/tests/stress.cc
SAN_OPT  := -O1 -g -fno-omit-frame-pointer
ASAN_FL  := -fsanitize=address,undefined -fno-sanitize-recover=undefined
TSAN_FL  := -fsanitize=thread
$(BUILD)/asan/%.o: csrc/%.cc
	@mkdir -p $(dir $@)
	$(CXX) $(CPPFLAGS) $(CXXSTD) $(SAN_OPT) $(HOSTARCH) -pthread $(ASAN_FL) -MMD -MP -c $< -o $@
$(BUILD)/tsan/%.o: csrc/%.cc
	@mkdir -p $(dir $@)
	$(CXX) $(CPPFLAGS) $(CXXSTD) $(SAN_OPT) $(HOSTARCH) -pthread $(TSAN_FL) -MMD -MP -c $< -o $@
$(BUILD)/plain/%.o: csrc/%.cc
	@mkdir -p $(dir $@)
	$(CXX) $(CPPFLAGS) $(CXXSTD) -O2 -g $(HOSTARCH) -pthread -MMD -MP -c $< -o $@
$(BUILD)/asan/stress: $(patsubst csrc/%.cc,$(BUILD)/asan/%.o,$(SAN_SRCS))
	$(CXX) -pthread $(ASAN_FL) -o $@ $^ $(LDLIBS)
$(BUILD)/tsan/stress: $(patsubst csrc/%.cc,$(BUILD)/tsan/%.o,$(SAN_SRCS))
	$(CXX) -pthread $(TSAN_FL) -o $@ $^ $(LDLIBS)
$(BUILD)/plain/stress: $(patsubst csrc/%.cc,$(BUILD)/plain/%.o,$(SAN_SRCS))
	$(CXX) -pthread -o $@ $^ $(LDLIBS)
asan: $(BUILD)/asan/stress
	ASAN_OPTIONS=detect_leaks=1 $(BUILD)/asan/stress
tsan: $(BUILD)/tsan/stress
	TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" $(BUILD)/tsan/stress
stress: $(BUILD)/plain/stress
	$(BUILD)/plain/stress 3

-include $(patsubst csrc/%.cc,$(BUILD)/asan/%.d,$(SAN_SRCS)) $(patsubst csrc/%.cc,$(BUILD)/tsan/%.d,$(SAN_SRCS)) \
  $(patsubst csrc/%.cc,$(BUILD)/plain/%.d,$(SAN_SRCS))

clean:
	rm -rf $(BUILD) $(EXT) $(TOOL_BINS)

-include $(CORE_OBJS:.o=.d) $(GPU_OBJS:.o=.d) $(PY_OBJS:.o=.d) $(wildcard $(BUILD)/tools/*.d)
