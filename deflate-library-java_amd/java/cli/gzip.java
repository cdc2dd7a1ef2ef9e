/*
 * `java gzip InputFile OutputFile.gz` on the GPU codec: the reference CLI's behaviour
 * (S/gzip.java:25-79 -- argument checks and messages, GzipMetadata from the input file, exit status 1
 * with the message on stderr, the two speed lines) with io.nayuki.deflate.gpu.GzipOutputStream
 * underneath.  Same output bytes as the reference (RLE_DYNAMIC, 64 KiB blocks, FHCRC + FNAME).
 */
import java.io.File;
import java.io.FileInputStream;
import java.io.FileOutputStream;
import java.io.IOException;
import java.io.InputStream;
import java.io.OutputStream;
import java.util.Optional;
import io.nayuki.deflate.GzipMetadata;
import io.nayuki.deflate.gpu.GzipOutputStream;


public final class gzip {
	
	public static void main(String[] args) {
		String err = run(args);
		if (err == null)
			return;
		System.err.println(err);
		System.exit(1);
	}
	
	
	// null on success, else the message the reference prints
	private static String run(String[] args) {
		if (args.length != 2)
			return "Usage: java gzip InputFile OutputFile.gz";
		var src = new File(args[0]);
		var dst = new File(args[1]);
		String bad = !src.exists() ? "Input path does not exist: " + src
			: src.isDirectory() ? "Input path is a directory: " + src
			: dst.isDirectory() ? "Output path is a directory: " + dst : null;
		if (bad != null)
			return bad;
		
		int mtime = (int)(src.lastModified() / 1000);            // 0: no timestamp
		var meta = new GzipMetadata(GzipMetadata.CompressionMethod.DEFLATE, false,
			mtime == 0 ? Optional.empty() : Optional.of(mtime), 0, GzipMetadata.OperatingSystem.UNIX,
			Optional.empty(), Optional.of(src.getName()), Optional.empty(), true);
		
		long t0 = System.nanoTime();
		try (InputStream in = new FileInputStream(src);
				OutputStream out = new GzipOutputStream(new FileOutputStream(dst), meta)) {
			in.transferTo(out);
		} catch (IOException e) {
			return "I/O exception: " + e.getMessage();
		}
		double secs = (System.nanoTime() - t0) / 1.0e9;
		System.err.printf("Input  speed: %.2f MB/s%n", src.length() / 1e6 / secs);
		System.err.printf("Output speed: %.2f MB/s%n", dst.length() / 1e6 / secs);
		return null;
	}
	
}
