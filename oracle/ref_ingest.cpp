// ref_ingest.cpp — TEST INFRASTRUCTURE ONLY (part of oracle/).
//
// Drives the *real* reference capture readers (Pcap++/src/PcapFileDevice.cpp + 3rdParty/LightPcapNg,
// compiled from /root/reference by oracle/Makefile into oracle/_ref/libpcpp_ref.so, without libpcap) so
// the engine's ingest (pcppx_pcap_*) can be checked record for record. The device is picked from the
// file's first bytes, as IFileReaderDevice::createReader does (PcapFileDevice.cpp:546-583), except that
// the Kuznetzov "modified" pcap magics (which createReader rejects) go to PcapFileReaderDevice as
// getReader does for a .pcap name (:533-544).
//
// ref_read_capture(path, ...) reads every packet with getNextPacket(RawPacket&) and writes, per packet,
// the captured bytes (back to back), caplen, frame length, timestamp (ns) and link type. Returns the
// packet count, -1 if the device does not open, -2 if a capacity is exceeded (call again larger).
#include "PcapFileDevice.h"
#include "RawPacket.h"
#include "Logger.h"

#include <cstdint>
#include <cstring>
#include <fstream>
#include <memory>

extern "C" int ref_read_capture(const char* path, uint8_t* data, uint64_t data_cap, uint32_t* caplens,
                                uint32_t* frame_lens, uint64_t* ts_ns, uint32_t* linktypes, uint32_t max_packets,
                                uint64_t* bytes_out)
{
	pcpp::Logger::getInstance().suppressLogs();
	uint32_t magic = 0;
	{
		std::ifstream f(path, std::ios::binary);
		if (!f)
			return -1;
		f.read(reinterpret_cast<char*>(&magic), 4);
		if (f.gcount() != 4)
			return -1;
	}
	std::unique_ptr<pcpp::IFileReaderDevice> reader;
	switch (magic)
	{
	case 0xa1b2c3d4: case 0xd4c3b2a1: case 0xa1b2cd34: case 0x34cdb2a1: case 0xa1b23c4d: case 0x4d3cb2a1:
		reader.reset(new pcpp::PcapFileReaderDevice(path));
		break;
	case 0x0A0D0D0A:
		reader.reset(new pcpp::PcapNgFileReaderDevice(path));
		break;
	default:
		return -1;
	}
	if (!reader->open())
		return -1;
	pcpp::RawPacket raw;
	uint32_t n = 0;
	uint64_t used = 0;
	while (reader->getNextPacket(raw))
	{
		const uint32_t cap = (uint32_t)raw.getRawDataLen();
		if (n >= max_packets || used + cap > data_cap)
		{
			reader->close();
			return -2;
		}
		if (cap)
			std::memcpy(data + used, raw.getRawData(), cap);
		caplens[n] = cap;
		frame_lens[n] = (uint32_t)raw.getFrameLength();
		const timespec ts = raw.getPacketTimeStamp();
		ts_ns[n] = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
		linktypes[n] = (uint32_t)raw.getLinkLayerType();
		used += cap;
		++n;
	}
	reader->close();
	*bytes_out = used;
	return (int)n;
}
