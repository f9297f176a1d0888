# Builds the MI355X (gfx950) CRC32C engine and its C-ABI:
#   libhdfs3_amd/lib/libhdfs3_crc.so      product (include/hdfs3_crc.h, hdfs3_client.h, hdfs3_hdfs.h);
#                                         exports only the C API (libhdfs3_crc.map)
#   libhdfs3_amd/lib/libhdfs3_crc_lab.so  measurement library for tools/ and the A/B tests: the
#                                         same sources with HDFS3_LAB=1 (kernel-variant knob,
#                                         experiment kernels, read-ceiling kernels, hdfs3x_*)
# plus test infrastructure (loopback datanode, native consumers) and the oracle (oracle/Makefile).
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CSRC     := libhdfs3_amd/csrc
LIBDIR   := libhdfs3_amd/lib
OBJDIR   := build/obj
LABDIR   := build/obj_lab
HIPFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Iinclude -I$(CSRC)
HOSTFLAGS:= -O3 -std=c++17 -fPIC -Wall -Iinclude -I$(CSRC)

LIB      := $(LIBDIR)/libhdfs3_crc.so
LABLIB   := $(LIBDIR)/libhdfs3_crc_lab.so
LOOPBACK := $(LIBDIR)/libhdfs3_loopback.so

# device/HIP translation units (built twice: product and lab), host-only ones (shared)
HIP_SRCS := crc32c_kernels.hip hdfs3_crc.cpp multi_device.cpp numa.cpp client/block_reader.cpp client/input_stream.cpp \
            client/output_stream.cpp client/local_reader.cpp client/block_checksum.cpp client/pipeline.cpp
HOST_SRCS:= host_crc32c.cpp client/wire.cpp client/net.cpp md5.cpp client/hdfs_shim.cpp
objname   = $(subst /,_,$(basename $(1))).o
HIP_OBJS := $(foreach s,$(HIP_SRCS),$(OBJDIR)/$(call objname,$(s)))
LAB_OBJS := $(foreach s,$(HIP_SRCS),$(LABDIR)/$(call objname,$(s))) $(LABDIR)/crc32c_experiments.o
HOST_OBJS:= $(foreach s,$(HOST_SRCS),$(OBJDIR)/$(call objname,$(s)))
HDRS     := $(wildcard include/*.h) $(wildcard $(CSRC)/*.h) $(wildcard $(CSRC)/client/*.h)

CONSUMER := tests/native/abi_consumer
CLIENT_CONSUMER := tests/native/client_consumer
HDFS_CONSUMER := tests/native/hdfs_consumer

# Adapters of integration/ compiled against the reference's OWN headers (and, for the block
# reader, linked with the reference's src/common/Exception.cpp, which builds from that one
# file): only where /root/reference exists; outputs go to oracle/_ref/ and travel with the tree.
REF      ?= /root/reference
REFBIN   := oracle/_ref
REFCHECK := $(if $(wildcard $(REF)/src/common/Checksum.h),$(REFBIN)/checksum_kat $(REFBIN)/blockreader_consumer,)

all: $(LIB) $(LABLIB) $(LOOPBACK) oracle $(CONSUMER) $(CLIENT_CONSUMER) $(HDFS_CONSUMER) $(REFCHECK)

define hip_rule
$(OBJDIR)/$(call objname,$(1)): $(CSRC)/$(1) $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $$< -o $$@
$(LABDIR)/$(call objname,$(1)): $(CSRC)/$(1) $(HDRS)
	@mkdir -p $(LABDIR)
	$(HIPCC) $(HIPFLAGS) -DHDFS3_LAB=1 -x hip -c $$< -o $$@
endef
$(foreach s,$(HIP_SRCS),$(eval $(call hip_rule,$(s))))

$(LABDIR)/crc32c_experiments.o: $(CSRC)/crc32c_experiments.hip $(HDRS)
	@mkdir -p $(LABDIR)
	$(HIPCC) $(HIPFLAGS) -DHDFS3_LAB=1 -c $< -o $@

define host_rule
$(OBJDIR)/$(call objname,$(1)): $(CSRC)/$(1) $(HDRS)
	@mkdir -p $(OBJDIR)
	g++ $(HOSTFLAGS) -c $$< -o $$@
endef
$(foreach s,$(HOST_SRCS),$(eval $(call host_rule,$(s))))

$(LIB): $(HIP_OBJS) $(HOST_OBJS) $(CSRC)/libhdfs3_crc.map
	@mkdir -p $(LIBDIR)
	$(HIPCC) -shared --offload-arch=$(ARCH) -Wl,--version-script=$(CSRC)/libhdfs3_crc.map -o $@ $(HIP_OBJS) $(HOST_OBJS)

$(LABLIB): $(LAB_OBJS) $(HOST_OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(LAB_OBJS) $(HOST_OBJS)

# test/bench infrastructure: loopback datanode (tools/loopback)
$(LOOPBACK): tools/loopback/loopback_datanode.cpp $(OBJDIR)/client_wire.o $(OBJDIR)/client_net.o $(OBJDIR)/md5.o
	@mkdir -p $(LIBDIR)
	g++ $(HOSTFLAGS) -shared -pthread -o $@ tools/loopback/loopback_datanode.cpp $(OBJDIR)/client_wire.o $(OBJDIR)/client_net.o $(OBJDIR)/md5.o

# test infrastructure: a C++ consumer of the C-ABI, checked against the oracle
$(OBJDIR)/consumer_oracle.o: oracle/crc32c_oracle.c oracle/crc32c_oracle.h
	@mkdir -p $(OBJDIR)
	gcc -O2 -msse4.2 -mpclmul -c $< -o $@

$(CONSUMER): tests/native/abi_consumer.cpp include/hdfs3_crc.h $(OBJDIR)/consumer_oracle.o $(LIB)
	g++ -O2 -std=c++17 -Wall -Iinclude -Ioracle -o $@ tests/native/abi_consumer.cpp $(OBJDIR)/consumer_oracle.o \
	    -L$(LIBDIR) -lhdfs3_crc -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath-link,/opt/rocm/lib -pthread

# test infrastructure: a C++ consumer of the client drop-ins (include/hdfs3_client.h) over the
# loopback datanode, in the reference function tests' shape
$(CLIENT_CONSUMER): tests/native/client_consumer.cpp include/hdfs3_client.h $(OBJDIR)/consumer_oracle.o $(LIB) $(LOOPBACK)
	g++ -O2 -std=c++17 -Wall -Iinclude -Ioracle -o $@ tests/native/client_consumer.cpp $(OBJDIR)/consumer_oracle.o \
	    -L$(LIBDIR) -lhdfs3_crc -lhdfs3_loopback -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath-link,/opt/rocm/lib \
	    -pthread

# test infrastructure: a plain C program on the hdfs.h surface (include/hdfs3_hdfs.h) over the
# loopback datanode: hdfsRead / hdfsPread / hdfsWrite exactly as a libhdfs3 caller writes them
$(HDFS_CONSUMER): tests/native/hdfs_consumer.c include/hdfs3_hdfs.h $(OBJDIR)/consumer_oracle.o $(LIB) $(LOOPBACK)
	gcc -O2 -std=c11 -Wall -Iinclude -Ioracle -o $@ tests/native/hdfs_consumer.c $(OBJDIR)/consumer_oracle.o \
	    -L$(LIBDIR) -lhdfs3_crc -lhdfs3_loopback -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath-link,/opt/rocm/lib \
	    -pthread

$(REFBIN)/checksum_kat: tests/native/checksum_kat.cpp integration/GpuCrc32c.h include/hdfs3_crc.h $(LIB)
	@mkdir -p $(REFBIN)
	g++ -O2 -std=c++17 -Wall -Iinclude -Iintegration -I$(REF)/src/common -o $@ tests/native/checksum_kat.cpp \
	    -L$(LIBDIR) -lhdfs3_crc -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath-link,/opt/rocm/lib -pthread

$(REFBIN)/blockreader_consumer: tests/native/blockreader_consumer.cpp integration/GpuRemoteBlockReader.h \
                                $(OBJDIR)/consumer_oracle.o $(LIB) $(LOOPBACK)
	@mkdir -p $(REFBIN)
	g++ -O2 -std=c++17 -Wall -Iinclude -Iintegration -Ioracle -I$(REF)/src/client -I$(REF)/src/common -o $@ \
	    tests/native/blockreader_consumer.cpp $(REF)/src/common/Exception.cpp $(OBJDIR)/consumer_oracle.o \
	    -L$(LIBDIR) -lhdfs3_crc -lhdfs3_loopback -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' \
	    -Wl,-rpath-link,/opt/rocm/lib -pthread

oracle:
	$(MAKE) -C oracle all
	@if [ -d /root/reference/src/common ]; then $(MAKE) -C oracle ref; fi

clean:
	rm -rf build $(LIB) $(LABLIB) $(LOOPBACK) $(CONSUMER) $(CLIENT_CONSUMER) $(HDFS_CONSUMER)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
