# Builds the MI355X (gfx950) CRC32C engine and its C-ABI:
#   libhdfs3_amd/lib/libhdfs3_crc.so   (include/hdfs3_crc.h)
# and the test-only oracle (oracle/Makefile).
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CSRC     := libhdfs3_amd/csrc
LIBDIR   := libhdfs3_amd/lib
OBJDIR   := build/obj
HIPFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Iinclude -I$(CSRC)
HOSTFLAGS:= -O3 -std=c++17 -fPIC -Wall -Iinclude -I$(CSRC)

LIB      := $(LIBDIR)/libhdfs3_crc.so
LOOPBACK := $(LIBDIR)/libhdfs3_loopback.so
OBJS     := $(OBJDIR)/crc32c_kernels.o $(OBJDIR)/crc32c_experiments.o $(OBJDIR)/hdfs3_crc.o $(OBJDIR)/host_crc32c.o \
            $(OBJDIR)/client_wire.o $(OBJDIR)/client_net.o $(OBJDIR)/client_block_reader.o \
            $(OBJDIR)/client_input_stream.o $(OBJDIR)/client_output_stream.o \
            $(OBJDIR)/client_local_reader.o $(OBJDIR)/client_block_checksum.o $(OBJDIR)/md5.o

CONSUMER := tests/native/abi_consumer
CLIENT_CONSUMER := tests/native/client_consumer

all: $(LIB) $(LOOPBACK) oracle $(CONSUMER) $(CLIENT_CONSUMER)

$(OBJDIR)/crc32c_kernels.o: $(CSRC)/crc32c_kernels.hip $(CSRC)/crc32c_device.h $(CSRC)/crc32c_kernels.h $(CSRC)/crc32c_tables.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/crc32c_experiments.o: $(CSRC)/crc32c_experiments.hip $(CSRC)/crc32c_device.h $(CSRC)/crc32c_kernels.h $(CSRC)/crc32c_tables.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/hdfs3_crc.o: $(CSRC)/hdfs3_crc.cpp include/hdfs3_crc.h $(CSRC)/crc32c_kernels.h $(CSRC)/crc32c_tables.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(OBJDIR)/host_crc32c.o: $(CSRC)/host_crc32c.cpp $(CSRC)/crc32c_tables.h
	@mkdir -p $(OBJDIR)
	g++ $(HOSTFLAGS) -c $< -o $@

$(OBJDIR)/client_wire.o: $(CSRC)/client/wire.cpp $(CSRC)/client/wire.h
	@mkdir -p $(OBJDIR)
	g++ $(HOSTFLAGS) -c $< -o $@

$(OBJDIR)/client_net.o: $(CSRC)/client/net.cpp $(CSRC)/client/net.h
	@mkdir -p $(OBJDIR)
	g++ $(HOSTFLAGS) -c $< -o $@

$(OBJDIR)/client_block_reader.o: $(CSRC)/client/block_reader.cpp $(CSRC)/client/block_reader.h include/hdfs3_client.h include/hdfs3_crc.h $(CSRC)/ctx.h $(CSRC)/client/wire.h $(CSRC)/client/net.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(OBJDIR)/client_input_stream.o: $(CSRC)/client/input_stream.cpp $(CSRC)/client/block_reader.h include/hdfs3_client.h include/hdfs3_crc.h $(CSRC)/ctx.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(OBJDIR)/client_output_stream.o: $(CSRC)/client/output_stream.cpp include/hdfs3_client.h include/hdfs3_crc.h $(CSRC)/ctx.h $(CSRC)/client/wire.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(OBJDIR)/client_local_reader.o: $(CSRC)/client/local_reader.cpp include/hdfs3_client.h include/hdfs3_crc.h $(CSRC)/ctx.h $(CSRC)/client/wire.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(OBJDIR)/client_block_checksum.o: $(CSRC)/client/block_checksum.cpp include/hdfs3_client.h $(CSRC)/ctx.h $(CSRC)/client/wire.h $(CSRC)/client/net.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(OBJDIR)/md5.o: $(CSRC)/md5.cpp $(CSRC)/md5.h
	@mkdir -p $(OBJDIR)
	g++ $(HOSTFLAGS) -c $< -o $@

# test/bench infrastructure: loopback datanode (tools/loopback)
$(LOOPBACK): tools/loopback/loopback_datanode.cpp $(OBJDIR)/client_wire.o $(OBJDIR)/client_net.o $(OBJDIR)/md5.o
	@mkdir -p $(LIBDIR)
	g++ $(HOSTFLAGS) -shared -pthread -o $@ tools/loopback/loopback_datanode.cpp $(OBJDIR)/client_wire.o $(OBJDIR)/client_net.o $(OBJDIR)/md5.o

$(LIB): $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJS)

# test infrastructure: a C++ consumer of the C-ABI, checked against the oracle
$(CONSUMER): tests/native/abi_consumer.cpp include/hdfs3_crc.h oracle/crc32c_oracle.c oracle/crc32c_oracle.h $(LIB)
	gcc -O2 -msse4.2 -mpclmul -c oracle/crc32c_oracle.c -o $(OBJDIR)/consumer_oracle.o
	g++ -O2 -std=c++17 -Wall -Iinclude -Ioracle -o $@ tests/native/abi_consumer.cpp $(OBJDIR)/consumer_oracle.o \
	    -L$(LIBDIR) -lhdfs3_crc -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath-link,/opt/rocm/lib -pthread

# test infrastructure: a C++ consumer of the client drop-ins (include/hdfs3_client.h) over the
# loopback datanode, in the reference function tests' shape
$(CLIENT_CONSUMER): tests/native/client_consumer.cpp include/hdfs3_client.h $(CONSUMER) $(LIB) $(LOOPBACK)
	g++ -O2 -std=c++17 -Wall -Iinclude -Ioracle -o $@ tests/native/client_consumer.cpp $(OBJDIR)/consumer_oracle.o \
	    -L$(LIBDIR) -lhdfs3_crc -lhdfs3_loopback -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath-link,/opt/rocm/lib \
	    -pthread

oracle:
	$(MAKE) -C oracle all
	@if [ -d /root/reference/src/common ]; then $(MAKE) -C oracle ref; fi

clean:
	rm -rf build $(LIB) $(LOOPBACK) $(CONSUMER) $(CLIENT_CONSUMER)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
